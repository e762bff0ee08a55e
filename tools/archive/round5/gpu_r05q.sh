#!/bin/bash
# Round-5 GPU batch q: LightGlue attention with the score MFMAs as inline asm writing VGPRs
# and Q in the accumulator file (tree) vs the builtin form (ab_att/a0): kernel + LightGlue
# GPU tests, attention determinism across shapes (both arms), LightGlue stage bench digest
# + time ABAB.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_lightglue_gpu.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > "$O/r05q_pytest.log" 2>&1
rc=$?; tail -3 "$O/r05q_pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/attn_det_probe.py multi-level-indoor-slam_amd/mlgate > "$O/r05q_det_tree.log" 2>&1 \
  || { tail -5 "$O/r05q_det_tree.log"; exit 1; }
tail -3 "$O/r05q_det_tree.log"
run() {  # tag, lib dir or "tree", command...
  local tag="$1" lib="$2"; shift 2
  local pre=""; [ "$lib" != tree ] && pre="tools/ab_run.py --lib-dir $lib"
  timeout -k 10 300 python -u $pre "$@" > "$O/r05q_$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$O/r05q_$tag.log"; exit 1; }
  echo "$tag $(grep '^{' "$O/r05q_$tag.log" | tail -1 | cut -c1-700)"
}
for rep in 0 1; do
  run lg_tree_$rep tree tools/lg_bench.py --pairs 2048 --iters 2
  run lg_a0_$rep ab_att/a0 tools/lg_bench.py --pairs 2048 --iters 2
done
