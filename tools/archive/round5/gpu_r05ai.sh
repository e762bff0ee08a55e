#!/bin/bash
# Round-5 GPU batch ai: k_asg_sim operand prefetch depth 2 (ab_asg/pf2, -DASG_PF=2) vs 1 (tree).
# general bounded loops only (ab_asg/pf2): LightGlue / SuperGlue / kernel GPU tests, LightGlue stage
# bench ABAB (digest), then rocprof kernel stats of the stage bench per arm (k_asg_arg average).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_lightglue_gpu.py tests/test_superglue_gpu.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > "$O/r05ai_pytest.log" 2>&1
rc=$?; tail -3 "$O/r05ai_pytest.log"; [ $rc -eq 0 ] || exit $rc
run() {  # tag, lib dir or "tree", command...
  local tag="$1" lib="$2"; shift 2
  local pre=""; [ "$lib" != tree ] && pre="tools/ab_run.py --lib-dir $lib"
  timeout -k 10 300 python -u $pre "$@" > "$O/r05ai_$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$O/r05ai_$tag.log"; exit 1; }
  echo "$tag $(grep '^{' "$O/r05ai_$tag.log" | tail -1 | cut -c1-300)"
}
for rep in 0 1; do
  run lg_tree_$rep tree tools/lg_bench.py --pairs 2048 --iters 2
  run lg_pf2_$rep ab_asg/pf2 tools/lg_bench.py --pairs 2048 --iters 2
done
cd /tmp && export TMPDIR=/tmp
for arm in tree pf2; do
  pre=""; [ $arm != tree ] && pre="$R/tools/ab_run.py --lib-dir $R/ab_asg/pf2"
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ai_$arm -o run -- python3 $pre "$R/tools/lg_bench.py" --pairs 2048 --iters 2 \
      > "$O/r05ai_prof_$arm.log" 2>&1 || { echo "prof $arm failed"; tail -3 "$O/r05ai_prof_$arm.log"; exit 1; }
  f=$(find /tmp/ai_$arm -name '*kernel_stats.csv' | head -1)
  echo "== $arm"; grep -E "k_asg" "$f" | cut -c1-60,200-400 | head -5
  cp "$f" "$O/r05ai_stats_$arm.csv"
done
