#!/bin/bash
# Round-5 GPU batch h: attribution probes.  The fused FFN with one phase dropped per
# build (MLG_FFN_PROBE bits, tools/proj_pipe_check.py's ffn timing, 2 M tokens), and the
# 5-point RANSAC solver cut after each stage (RS_ABLATE) on bench-like pairs.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
run() {  # tag, lib dir or "tree", command...
  local tag="$1" lib="$2"; shift 2
  local pre=""; [ "$lib" != tree ] && pre="tools/ab_run.py --lib-dir $lib"
  timeout -k 10 240 python -u $pre "$@" > "$O/r05h_$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$O/r05h_$tag.log"; exit 1; }
  echo "$tag $(grep '^{' "$O/r05h_$tag.log" | tail -1 | cut -c1-600)"
}
for rep in 0 1; do
  run ffn_tree_$rep tree tools/proj_pipe_check.py --iters 10
  for b in 1 2 3 4 8 16 28 32 64; do run ffn_p${b}_$rep ab_ffnp/p$b tools/proj_pipe_check.py --iters 10; done
done
for rep in 0 1; do
  run rs_tree_$rep tree tools/ransac_bench.py --pairs 5000 --matches 600 --inliers 0.2 --reps 3
  for b in 1 2 3; do run rs_a${b}_$rep ab_rs/a$b tools/ransac_bench.py --pairs 5000 --matches 600 --inliers 0.2 --reps 3; done
done
# the per-lane null space (MLG_RS_NULL_SPLIT) against the in-group QR: digest + time
for rep in 0 1; do
  run rs_null_tree_$rep tree tools/ransac_bench.py --pairs 5000 --matches 600 --inliers 0.2 --reps 3
  run rs_null_n0_$rep ab_rs/n0 tools/ransac_bench.py --pairs 5000 --matches 600 --inliers 0.2 --reps 3
  run rs_null_tree_hi_$rep tree tools/ransac_bench.py --pairs 2000 --matches 1200 --inliers 0.5 --reps 3
  run rs_null_n0_hi_$rep ab_rs/n0 tools/ransac_bench.py --pairs 2000 --matches 1200 --inliers 0.5 --reps 3
done
