#!/bin/bash
# Round 6: the LoFTR pair group's split similarity as one batched persistent GEMM launch.
# (1) LoFTR GPU tests on the tree; (2) same-box ABAB tree vs ab/lfsim (-DMLG_LF_SIM_BATCH=0:
# one launch per pair) at 480x640 and 540x720 (digests must be equal: same tiles, same
# arithmetic); (3) the ViT's split GEMMs (the same kernel, nb = 1) tree vs ab/rev_head (the
# previous gemm_bf16.hip): time and descriptor digest; (4) rocprof of the tree at 540x720.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"; T="${1:-r06o}"
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_loftr_gpu.py tests/test_vit_gpu.py -x -q --timeout 300 --timeout-method thread > "$O/${T}_tests.log" 2>&1
rc=$?; tail -2 "$O/${T}_tests.log"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh ab/lfsim ${T}_640 2 -- tools/loftr_bench.py --frames 64 --pairs 64 --iters 4 || exit 1
bash tools/gpu_ab.sh ab/lfsim ${T}_isec 2 -- tools/loftr_bench.py --frames 64 --pairs 64 --iters 4 --hw 540x720 || exit 1
bash tools/gpu_ab.sh ab/rev_head ${T}_vit 2 -- tools/vit_bench.py --frames 492 --batch 246 --iters 3 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/${T}_prof -o run -- \
    python3 -u "$R/tools/loftr_bench.py" --frames 64 --pairs 64 --iters 2 --hw 540x720 > "$O/${T}_prof.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 "$O/${T}_prof.log"; exit $rc; }
find /tmp/${T}_prof -name '*kernel_stats.csv' -exec cp {} "$O/${T}_kernel_stats.csv" \;
echo done
