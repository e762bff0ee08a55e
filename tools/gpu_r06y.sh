#!/bin/bash
# Round 6: LoFTR FPN merge fused into the lateral 1x1 conv epilogue (EpiConvUp)
# (tree) vs the conv + k_lf_up_add (ab/fpn, -DMLG_LF_FPN_FUSED=0): LoFTR GPU tests (incl. the
# sharded gate case) on the tree, then same-box ABAB of tools/loftr_bench.py at 480x640 and
# 540x720 (digests must be equal) and the bench's LoFTR sub-object.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"; T="${1:-r06y}"
cd "$R"
timeout -k 10 500 python -u -m pytest tests/test_loftr_gpu.py tests/test_distributed_gpu.py -k "loftr or LoFTR or isec or split or backbone or matching or dropin" -x -q --timeout 300 --timeout-method thread > "$O/${T}_tests.log" 2>&1
rc=$?; tail -2 "$O/${T}_tests.log"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh ab/fpn ${T}_640 2 -- tools/loftr_bench.py --frames 64 --pairs 64 --iters 4 || exit 1
bash tools/gpu_ab.sh ab/fpn ${T}_isec 2 -- tools/loftr_bench.py --frames 64 --pairs 64 --iters 4 --hw 540x720 || exit 1
