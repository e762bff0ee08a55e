#!/bin/bash
# r04m: LoFTR values / L in the qkv epilogue, parallel column-stat merge; LoFTR tests and
# profile; attributed PMC of the LightGlue stage and the split-bf16 ViT
set -u
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_loftr_gpu.py "tests/test_distributed_gpu.py::test_sharded_gate_equals_single_rank[loftr]" > gpurun_out/r04m_loftr.log 2>&1 && echo "loftr tests ok" &&
{ cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; } &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04m_lfprof -o lf -- python3 tools/loftr_bench.py --pairs 64 > gpurun_out/r04m_loftr_bench.log 2>&1 && echo "loftr prof ok" &&
timeout -k 10 900 bash tools/pmc_kernels.sh r04m > gpurun_out/r04m_pmc.log 2>&1 && echo "pmc ok"
rc=$?
echo "rc=$rc"
tail -3 gpurun_out/r04m_loftr.log; grep '^{' gpurun_out/r04m_loftr_bench.log; tail -5 gpurun_out/r04m_pmc.log
exit $rc
