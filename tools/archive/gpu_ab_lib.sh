#!/bin/bash
# HISTORICAL (kept as the recipe of the profiles it produced): it switches arms through
# runtime knobs (MLG_FFN_* / MLG_PROJ_* / MLG_GEMM_VARIANT env vars, MLGATE_LIB_DIR) that the
# library no longer reads, so both arms would now run the same build.  Build each arm
# with -D flags instead and load it through tools/ab_run.py --lib-dir (tools/gpu_r03ag.sh).
echo "$0: historical recipe; its runtime A/B knobs are gone (see header)" >&2; exit 2
# Same-box A/B of two builds: ab_old/ (baseline libraries, loaded through MLGATE_LIB_DIR)
# against the in-tree build.  Parity tests ($AB_TESTS) on the in-tree build first, then
# the bench, alternating arms ($AB_ROUNDS rounds).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${AB_TESTS:-tests/test_superpoint_gpu.py} -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ab_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in $(seq 1 ${AB_ROUNDS:-1}); do
for arm in new old; do
  if [ $arm = old ]; then export MLGATE_LIB_DIR=$PWD/ab_old; else unset MLGATE_LIB_DIR; fi
  timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_bench_$arm$i.log 2>&1
  rc=$?; echo "bench $arm rc=$rc"; tail -1 gpurun_out/ab_bench_$arm$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['stage_ms_per_step'], d['config']['false_loop_closure_rejections']['total'])"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
done
