#!/bin/bash
# Same-box A/B: DeviceGate RANSAC on a side stream (MLGATE_RANSAC_SIDE=1, default) vs the
# main stream; the full-gate GPU test first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/side_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/side_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 0 1 0; do
  MLGATE_RANSAC_SIDE=$r timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/side_bench_$r.log 2>&1
  rc=$?; echo "bench side=$r rc=$rc"; tail -1 gpurun_out/side_bench_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['false_loop_closure_rejections'])"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
