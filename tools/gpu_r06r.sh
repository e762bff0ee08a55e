#!/bin/bash
# Round 6: k_conv256's staged epilogue (tree) vs the fragment-at-a-time one (ab/convold,
# -DMLG_CONV_STAGED=0): LoFTR GPU tests on the tree, then same-box ABAB of
# tools/loftr_bench.py at 480x640 and 540x720 (digests must be equal).  The timing probe
# that motivated it (epilogue skipped, results invalid) was ab/convprobe.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"; T="${1:-r06s}"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_loftr_gpu.py -x -q --timeout 300 --timeout-method thread > "$O/${T}_tests.log" 2>&1
rc=$?; tail -2 "$O/${T}_tests.log"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh ab/convold ${T}_640 2 -- tools/loftr_bench.py --frames 64 --pairs 64 --iters 4 || exit 1
bash tools/gpu_ab.sh ab/convold ${T}_isec 2 -- tools/loftr_bench.py --frames 64 --pairs 64 --iters 4 --hw 540x720 || exit 1
