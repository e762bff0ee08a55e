#!/bin/bash
# LightGlue fixed-shift attention: kernel + matcher parity tests, then the stage microbench
# with the fixed shift and with the online max (A/B), then rocprof kernel stats.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/attn
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_lightglue_gpu.py tests/test_verify_gpu.py tests/test_pipeline_gpu.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/attn/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/attn/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/lg_bench.py --pairs 1024 --frames 128 || exit $?
timeout -k 10 300 python tools/lg_bench.py --pairs 1024 --frames 128 --online || exit $?
