#!/bin/bash
# r03ae: measured tolerances (LightGlue / SuperGlue vs fp32, verifier inliers vs the fp32 chain) + full suite after the FFN change
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_lightglue_gpu.py tests/test_superglue_gpu.py tests/test_pipeline_gpu.py -q -s -k "fp32 or verification_and_gate" --timeout 300 --timeout-method thread > gpurun_out/r03ae_tol.log 2>&1; rc=$?
grep -E "fp32|valid pairs|passed|failed" gpurun_out/r03ae_tol.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r03ae_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03ae_pytest.log; exit $rc
