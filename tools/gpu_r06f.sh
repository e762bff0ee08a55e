#!/bin/bash
# Round 6: per-kernel RANSAC times, round-5 build (contraction on; ab/rs_old) vs the tree
# (-ffp-contract=off, the Aberth complex products as explicit fma in both twins), rocprofv3
# kernel stats of tools/ransac_bench.py; the bit-exact RANSAC tests first.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_ransac_gpu.py -x -q --timeout 300 --timeout-method thread > "$O/r06f_pytest.log" 2>&1
rc=$?; tail -1 "$O/r06f_pytest.log"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for arm in tree rs_old; do
  if [ $arm = tree ]; then pre=""; else pre="$R/tools/ab_run.py --lib-dir $R/ab/rs_old"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rsp_$arm -o run -- \
      python3 $pre "$R/tools/ransac_bench.py" --pairs 5000 --matches 600 --inliers 0.2 > "$O/r06f_$arm.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 "$O/r06f_$arm.log"; exit $rc; }
  f=$(find /tmp/rsp_$arm -name '*kernel_stats.csv' | head -1)
  cp "$f" "$O/r06f_rocprof_ransac_$arm.csv"
  echo "== $arm"; grep -i ransac "$f" | cut -d, -f1-4 | cut -c1-160
done
