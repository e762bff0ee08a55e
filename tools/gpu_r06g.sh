#!/bin/bash
# Round 6 LoFTR A/B: the tree vs an arm built by tools/ab_build.sh (default ab/lf3: the
# two-read dual softmax against -DMLG_LF_TWO_READ=0; r06n: fast softmax-sum exp against
# -DMLG_LF_FAST_EXP=0 in ab/lfexp).  tools/gpu_r06g.sh TAG [AB_DIR].  LoFTR GPU tests on the tree, same-box ABAB of tools/loftr_bench.py at 480x640 and at the
# ISEC 540x720 (digest: counts + keypoints + conf; kdigest: counts + keypoints), then the
# per-kernel time of both arms at 540x720 under rocprofv3.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"; T="${1:-r06g}"; AB="${2:-ab/lf3}"
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_loftr_gpu.py -x -q --timeout 300 --timeout-method thread > "$O/${T}_loftr_tests.log" 2>&1
rc=$?; tail -2 "$O/${T}_loftr_tests.log"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh $AB ${T}_640 2 -- tools/loftr_bench.py --frames 64 --pairs 64 --iters 4 || exit 1
bash tools/gpu_ab.sh $AB ${T}_isec 2 -- tools/loftr_bench.py --frames 64 --pairs 64 --iters 4 --hw 540x720 || exit 1
cd /tmp && export TMPDIR=/tmp
for arm in tree ab; do
  if [ $arm = tree ]; then pre=""; else pre="$R/tools/ab_run.py --lib-dir $R/$AB"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/${T}_$arm -o run -- \
      python3 -u $pre "$R/tools/loftr_bench.py" --frames 64 --pairs 64 --iters 2 --hw 540x720 > "$O/${T}_prof_$arm.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 "$O/${T}_prof_$arm.log"; exit $rc; }
  find /tmp/${T}_$arm -name '*kernel_stats.csv' -exec cp {} "$O/${T}_kernel_stats_$arm.csv" \;
done
echo done
