#!/bin/bash
# Uninitialised-workspace check: every op's workspace filled with 0xFF bytes (NaN) first
# (MLG_WS_POISON=1); GPU parity tests and the bench's rejection count must not change.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
MLG_WS_POISON=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/poison_pytest.log 2>&1
rc=$?; echo "pytest poison rc=$rc $(tail -1 gpurun_out/poison_pytest.log)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/poison_pytest.log | head -20; fi
MLG_WS_POISON=1 timeout -k 10 400 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/poison_bench.log 2>&1
rc=$?; echo "bench poison rc=$rc"; tail -1 gpurun_out/poison_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['false_loop_closure_rejections'], d['config']['pairs_geometrically_valid'])"
exit $rc
