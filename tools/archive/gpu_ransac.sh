#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ransac_gpu.py tests/test_pipeline_gpu.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_ransac.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_ransac.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/ransac_bench.py
