#!/bin/bash
# GEMM-generation A/B on the GPU box: kernel parity tests, then per-kernel timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py ${EXTRA_TESTS:-} -q -x > gpurun_out/pytest_kernels.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -5 gpurun_out/pytest_kernels.log
if [ $rc -ne 0 ]; then exit $rc; fi
for b in ${GEMM_BATCHES:-64}; do
  timeout -k 10 300 python tools/gemm_bench.py --batch $b --variants ${GEMM_VARIANTS:-2,4} > gpurun_out/gemm_bench_$b.log 2>&1
  rc=$?; echo "gemm_bench batch $b rc=$rc"; grep '^{' gpurun_out/gemm_bench_$b.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
