#!/bin/bash
# (The MLGATE_LG_THREADS branch this script exercised was removed after the A/B; see profiles/r02r_ab_lightglue_threads.txt.)
# Same-box A/B: LightGlue chunks on 2 host threads / streams (MLGATE_LG_THREADS=2) vs 1;
# the full-gate GPU tests under both settings first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for t in 2 1; do
  MLGATE_LG_THREADS=$t timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/thr_pytest_$t.log 2>&1
  rc=$?; echo "pytest threads=$t rc=$rc $(tail -1 gpurun_out/thr_pytest_$t.log)"
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/thr_pytest_$t.log; exit $rc; fi
done
for t in ${AB_ARMS:-2 1 2 1}; do
  MLGATE_LG_THREADS=$t timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/thr_bench_$t.log 2>&1
  rc=$?; echo "bench threads=$t rc=$rc"; tail -1 gpurun_out/thr_bench_$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['stage_ms_per_step'], d['config']['false_loop_closure_rejections'], d['config']['pairs_geometrically_valid'])"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/thr_bench_$t.log; exit $rc; fi
done
