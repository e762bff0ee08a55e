#!/bin/bash
# r04l: LoFTR fused encoder tail + key-banded dual-softmax passes; whole GPU suite,
# LoFTR kernel profile, default bench
set -u
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_loftr_gpu.py "tests/test_distributed_gpu.py::test_sharded_gate_equals_single_rank[loftr]" > gpurun_out/r04l_loftr.log 2>&1 && echo "loftr tests ok" &&
timeout -k 10 600 $T -m gpu tests > gpurun_out/r04l_pytest_gpu.log 2>&1 && echo "suite ok" &&
{ cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; } &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04l_lfprof -o lf -- python3 tools/loftr_bench.py --pairs 64 > gpurun_out/r04l_loftr_bench.log 2>&1 && echo "loftr prof ok" &&
timeout -k 10 400 python -u bench.py > gpurun_out/r04l_bench.json 2> gpurun_out/r04l_bench.err && echo "bench ok"
rc=$?
echo "rc=$rc"
tail -3 gpurun_out/r04l_loftr.log; tail -2 gpurun_out/r04l_pytest_gpu.log; grep '^{' gpurun_out/r04l_loftr_bench.log
exit $rc
