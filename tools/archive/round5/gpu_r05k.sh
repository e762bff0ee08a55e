#!/bin/bash
# Round-5 GPU batch k: GELU polynomial as scalar v_fma_f32 chains (tree) vs packed f32
# (ab_gelupk, MLG_GELU_PK=1): FFN probe (sha1), LightGlue stage bench (digest), ViT
# forward (descriptor sha1), ABAB on one box; then the tree's FFN phase trace.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
run() {  # tag, lib dir or "tree", command...
  local tag="$1" lib="$2"; shift 2
  local pre=""; [ "$lib" != tree ] && pre="tools/ab_run.py --lib-dir $lib"
  timeout -k 10 300 python -u $pre "$@" > "$O/r05k_$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$O/r05k_$tag.log"; exit 1; }
  echo "$tag $(grep '^{' "$O/r05k_$tag.log" | tail -1 | cut -c1-700)"
}
for rep in 0 1; do
  run ffn_tree_$rep tree tools/proj_pipe_check.py --iters 10
  run ffn_pk_$rep ab_gelupk tools/proj_pipe_check.py --iters 10
done
for rep in 0 1; do
  run lg_tree_$rep tree tools/lg_bench.py --pairs 2048 --iters 2
  run lg_pk_$rep ab_gelupk tools/lg_bench.py --pairs 2048 --iters 2
done
for rep in 0 1; do
  run vit_tree_$rep tree tools/vit_bench.py
  run vit_pk_$rep ab_gelupk tools/vit_bench.py
done
# RANSAC: root-finder gathers through LDS (tree) vs 64-bit shuffles (ab_rs/l0)
for rep in 0 1; do
  run rs_tree_$rep tree tools/ransac_bench.py --pairs 5000 --matches 600 --inliers 0.2 --reps 3
  run rs_l0_$rep ab_rs/l0 tools/ransac_bench.py --pairs 5000 --matches 600 --inliers 0.2 --reps 3
  run rs_tree_hi_$rep tree tools/ransac_bench.py --pairs 2000 --matches 1200 --inliers 0.5 --reps 3
  run rs_l0_hi_$rep ab_rs/l0 tools/ransac_bench.py --pairs 2000 --matches 1200 --inliers 0.5 --reps 3
done
