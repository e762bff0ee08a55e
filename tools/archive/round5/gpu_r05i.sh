#!/bin/bash
# Round-5 GPU batch i: FFN co-resident workgroup stagger (MLG_FFN_STAGGER builds) on the
# 2 M-token probe and on the LightGlue stage bench (digest = bit-identity); the bench with
# the 5-point solver cut before its root finder (ab_rs/a1: decisions wrong, timing only)
# against the tree, to price RANSAC's share of the step while it overlaps LightGlue.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
run() {  # tag, lib dir or "tree", command...
  local tag="$1" lib="$2"; shift 2
  local pre=""; [ "$lib" != tree ] && pre="tools/ab_run.py --lib-dir $lib"
  timeout -k 10 300 python -u $pre "$@" > "$O/r05i_$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$O/r05i_$tag.log"; exit 1; }
  echo "$tag $(grep '^{' "$O/r05i_$tag.log" | tail -1 | cut -c1-700)"
}
for rep in 0 1; do
  run ffn_tree_$rep tree tools/proj_pipe_check.py --iters 10
  for v in s2m1 s4m1 s6m1 s4m2; do run ffn_${v}_$rep ab_ffns/$v tools/proj_pipe_check.py --iters 10; done
done
for rep in 0 1; do
  run lg_tree_$rep tree tools/lg_bench.py --pairs 2048 --iters 2
  for v in s4m1 s4m2; do run lg_${v}_$rep ab_ffns/$v tools/lg_bench.py --pairs 2048 --iters 2; done
done
for rep in 0 1; do
  run bench_tree_$rep tree bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --loftr-pairs 0
  run bench_rsa1_$rep ab_rs/a1 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --loftr-pairs 0
done
