#!/bin/bash
# GEMM-generation A/B on the GPU box: kernel parity tests, then per-kernel timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -x > gpurun_out/pytest_kernels.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -5 gpurun_out/pytest_kernels.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1
rc=$?; echo "gemm_bench rc=$rc"; cat gpurun_out/gemm_bench.log | grep '^{'
exit $rc
