#!/bin/bash
# Round-5 GPU batch aj: SuperPoint NMS with passes shrinking by their margin (tree, MLG_SP_NMS_MARGIN) vs
# every pass over the whole tile (ab_sp/m0): SuperPoint / pipeline GPU tests, sp_bench digest + time ABAB,
# rocprof k_sp_nms average per arm.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_superpoint_gpu.py tests/test_kernels_gpu.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > "$O/r05aj_pytest.log" 2>&1
rc=$?; tail -3 "$O/r05aj_pytest.log"; [ $rc -eq 0 ] || exit $rc
run() {  # tag, lib dir or "tree", command...
  local tag="$1" lib="$2"; shift 2
  local pre=""; [ "$lib" != tree ] && pre="tools/ab_run.py --lib-dir $lib"
  timeout -k 10 300 python -u $pre "$@" > "$O/r05aj_$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$O/r05aj_$tag.log"; exit 1; }
  echo "$tag $(grep '^{' "$O/r05aj_$tag.log" | tail -1 | cut -c1-300)"
}
for rep in 0 1; do
  run sp_tree_$rep tree tools/sp_bench.py
  run sp_m0_$rep ab_sp/m0 tools/sp_bench.py
done
cd /tmp && export TMPDIR=/tmp
for arm in tree m0; do
  pre=""; [ $arm != tree ] && pre="$R/tools/ab_run.py --lib-dir $R/ab_sp/m0"
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/aj_$arm -o run -- python3 $pre "$R/tools/sp_bench.py" \
      > "$O/r05aj_prof_$arm.log" 2>&1 || { echo "prof $arm failed"; tail -3 "$O/r05aj_prof_$arm.log"; exit 1; }
  f=$(find /tmp/aj_$arm -name '*kernel_stats.csv' | head -1)
  cp "$f" "$O/r05aj_stats_$arm.csv"; echo "stats $arm copied"
done
