#!/bin/bash
# Same-box A/B: LightGlue once per unordered pair (MLGATE_LG_DEDUP=1, default) vs once per
# ordered pair; the full-gate GPU tests first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py tests/test_verify_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dedup_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/dedup_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 0; do
  MLGATE_LG_DEDUP=$r timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/dedup_bench_$r.log 2>&1
  rc=$?; echo "bench dedup=$r rc=$rc"; tail -1 gpurun_out/dedup_bench_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c['pairs_verified'], c['pairs_matched_lightglue'], c['pairs_geometrically_valid'], c['false_loop_closure_rejections'])"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
