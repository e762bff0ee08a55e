#!/bin/bash
# Round 6: k_gemm256's row-staged epilogue for EpiConv (tree) vs fragment-at-a-time
# (ab/gemmrow, -DMLG_GEMM_ROW_STAGED=0); also the helper now shared with k_conv256.
# LoFTR + SuperGlue GPU tests on the tree, then same-box ABAB of tools/loftr_bench.py at
# 480x640 and 540x720 (digests must be equal) and of tools/sg_bench.py.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"; T="${1:-r06w}"
cd "$R"
timeout -k 10 500 python -u -m pytest tests/test_loftr_gpu.py tests/test_superglue_gpu.py -x -q --timeout 300 --timeout-method thread > "$O/${T}_tests.log" 2>&1
rc=$?; tail -2 "$O/${T}_tests.log"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh ab/gemmrow ${T}_640 2 -- tools/loftr_bench.py --frames 64 --pairs 64 --iters 4 || exit 1
bash tools/gpu_ab.sh ab/gemmrow ${T}_isec 2 -- tools/loftr_bench.py --frames 64 --pairs 64 --iters 4 --hw 540x720 || exit 1
bash tools/gpu_ab.sh ab/gemmrow ${T}_sg 1 -- tools/sg_bench.py || exit 1
