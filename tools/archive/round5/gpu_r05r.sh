#!/bin/bash
# Round-5 GPU batch r: LightGlue attention arms on the stage bench (digest + time), one box:
# tree = builtin score MFMAs (the product), pad = inline-asm VGPR scores forced to one
# workgroup per CU (dynamic LDS pad), a0pad = the product with the same pad (control)
# (the asm at two workgroups per CU ran 10 % slower: r05q).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
run() {  # tag, lib dir or "tree", command...
  local tag="$1" lib="$2"; shift 2
  local pre=""; [ "$lib" != tree ] && pre="tools/ab_run.py --lib-dir $lib"
  timeout -k 10 300 python -u $pre "$@" > "$O/r05r_$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$O/r05r_$tag.log"; exit 1; }
  echo "$tag $(grep '^{' "$O/r05r_$tag.log" | tail -1 | cut -c1-400)"
}
for rep in 0 1; do
  for arm in pad a0pad; do run lg_${arm}_$rep ab_att/$arm tools/lg_bench.py --pairs 2048 --iters 2; done
  run lg_tree_$rep tree tools/lg_bench.py --pairs 2048 --iters 2
done
