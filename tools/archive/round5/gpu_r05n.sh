#!/bin/bash
# Round-5 GPU batch n: LoFTR kv_part with LDS-staged whole-line k / v loads (tree) vs
# per-lane 16-B loads (ab_lf/kv0): LoFTR GPU tests, then loftr_bench digest + time ABAB.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_loftr_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
    > "$O/r05n_pytest.log" 2>&1
rc=$?; tail -3 "$O/r05n_pytest.log"; [ $rc -eq 0 ] || exit $rc
run() {  # tag, lib dir or "tree", command...
  local tag="$1" lib="$2"; shift 2
  local pre=""; [ "$lib" != tree ] && pre="tools/ab_run.py --lib-dir $lib"
  timeout -k 10 300 python -u $pre "$@" > "$O/r05n_$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$O/r05n_$tag.log"; exit 1; }
  echo "$tag $(grep '^{' "$O/r05n_$tag.log" | tail -1 | cut -c1-700)"
}
for rep in 0 1; do
  run lf_tree_$rep tree tools/loftr_bench.py --frames 64 --pairs 64
  run lf_kv0_$rep ab_lf/kv0 tools/loftr_bench.py --frames 64 --pairs 64
done
