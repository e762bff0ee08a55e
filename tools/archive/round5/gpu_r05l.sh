#!/bin/bash
# Round-5 GPU batch l: 5-point solver in 10-lane hypothesis groups (tree) vs 16-lane
# groups (ab_rs/g16): RANSAC GPU tests, then digest + time ABAB on bench-like pairs.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_ransac_gpu.py tests/test_decisions_gpu.py tests/test_bench_parity_gpu.py \
    tests/test_verify_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/r05l_pytest.log" 2>&1
rc=$?; tail -3 "$O/r05l_pytest.log"; [ $rc -eq 0 ] || exit $rc
run() {  # tag, lib dir or "tree", command...
  local tag="$1" lib="$2"; shift 2
  local pre=""; [ "$lib" != tree ] && pre="tools/ab_run.py --lib-dir $lib"
  timeout -k 10 300 python -u $pre "$@" > "$O/r05l_$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$O/r05l_$tag.log"; exit 1; }
  echo "$tag $(grep '^{' "$O/r05l_$tag.log" | tail -1 | cut -c1-700)"
}
for rep in 0 1; do
  run rs_tree_$rep tree tools/ransac_bench.py --pairs 5000 --matches 600 --inliers 0.2 --reps 3
  run rs_g16_$rep ab_rs/g16 tools/ransac_bench.py --pairs 5000 --matches 600 --inliers 0.2 --reps 3
  run rs_tree_hi_$rep tree tools/ransac_bench.py --pairs 2000 --matches 1200 --inliers 0.5 --reps 3
  run rs_g16_hi_$rep ab_rs/g16 tools/ransac_bench.py --pairs 2000 --matches 1200 --inliers 0.5 --reps 3
done
