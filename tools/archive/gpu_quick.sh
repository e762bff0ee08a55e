#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ransac_gpu.py tests/test_pipeline_gpu.py tests/test_superpoint_gpu.py tests/test_lightglue_gpu.py -m gpu -v -rf -s --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|fp32" gpurun_out/pytest_quick.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench_quick.log
exit $rc
