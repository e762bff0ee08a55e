#!/bin/bash
# Round-5 GPU batch m: the 5-point root finder in its own kernel (tree, MLG_RS_ROOTS_SPLIT)
# vs inside k_ransac_hyp5 (ab_rs/s0): RANSAC GPU tests, then digest + time ABAB.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_ransac_gpu.py tests/test_decisions_gpu.py tests/test_bench_parity_gpu.py \
    tests/test_verify_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/r05m_pytest.log" 2>&1
rc=$?; tail -3 "$O/r05m_pytest.log"; [ $rc -eq 0 ] || exit $rc
run() {  # tag, lib dir or "tree", command...
  local tag="$1" lib="$2"; shift 2
  local pre=""; [ "$lib" != tree ] && pre="tools/ab_run.py --lib-dir $lib"
  timeout -k 10 300 python -u $pre "$@" > "$O/r05m_$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$O/r05m_$tag.log"; exit 1; }
  echo "$tag $(grep '^{' "$O/r05m_$tag.log" | tail -1 | cut -c1-700)"
}
for rep in 0 1; do
  run rs_tree_$rep tree tools/ransac_bench.py --pairs 5000 --matches 600 --inliers 0.2 --reps 3
  run rs_s0_$rep ab_rs/s0 tools/ransac_bench.py --pairs 5000 --matches 600 --inliers 0.2 --reps 3
  run rs_tree_hi_$rep tree tools/ransac_bench.py --pairs 2000 --matches 1200 --inliers 0.5 --reps 3
  run rs_s0_hi_$rep ab_rs/s0 tools/ransac_bench.py --pairs 2000 --matches 1200 --inliers 0.5 --reps 3
done
