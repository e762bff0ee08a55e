#!/bin/bash
# LightGlue kernels: op-level + matcher parity tests, then the stage microbench (A/B of the
# projection kernels)
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_lightglue_gpu.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_lg.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_lg.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/lg_bench.py --pairs 1024 --frames 128 || exit $?
MLGATE_LG_PROJ_TILED=1 timeout -k 10 300 python tools/lg_bench.py --pairs 1024 --frames 128
