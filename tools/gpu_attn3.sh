#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/attn
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_lightglue_gpu.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/attn/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/attn/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for a in "" "--shifted"; do
  timeout -k 10 120 python tools/attn_bench.py --pairs 256 --len 2048 $a || exit $?
done
timeout -k 10 300 python tools/lg_bench.py --pairs 1024 --frames 128 || exit $?
timeout -k 10 300 python tools/lg_bench.py --pairs 1024 --frames 128 --online || exit $?
