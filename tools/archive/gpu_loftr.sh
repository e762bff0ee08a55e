#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/loftr
timeout -k 10 400 python -u -m pytest tests/test_loftr_gpu.py -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/loftr/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/loftr/pytest.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/loftr_bench.py || exit $?
