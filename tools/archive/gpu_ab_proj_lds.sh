#!/bin/bash
# HISTORICAL (kept as the recipe of the profiles it produced): it switches arms through
# runtime knobs (MLG_FFN_* / MLG_PROJ_* / MLG_GEMM_VARIANT env vars, MLGATE_LIB_DIR) that the
# library no longer reads, so both arms would now run the same build.  Build each arm
# with -D flags instead and load it through tools/ab_run.py --lib-dir (tools/gpu_r03ag.sh).
echo "$0: historical recipe; its runtime A/B knobs are gone (see header)" >&2; exit 2
# Same-box A/B of the LightGlue projection kernel: ab_old/ (baseline build, loaded through
# MLGATE_LIB_DIR) against the in-tree build; projection / LightGlue parity tests first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_lightglue_gpu.py tests/test_superglue_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/projlds_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/projlds_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for arm in new old new old; do
  if [ $arm = old ]; then export MLGATE_LIB_DIR=$PWD/ab_old; else unset MLGATE_LIB_DIR; fi
  timeout -k 10 120 python3 tools/proj_ab.py --iters 10 > gpurun_out/projlds_$arm.log 2>&1
  rc=$?; echo "$arm rc=$rc $(tail -1 gpurun_out/projlds_$arm.log | cut -c1-160)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
if [ "${AB_BENCH:-1}" = 1 ]; then
for arm in new old; do
  if [ $arm = old ]; then export MLGATE_LIB_DIR=$PWD/ab_old; else unset MLGATE_LIB_DIR; fi
  timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/projlds_bench_$arm.log 2>&1
  rc=$?; echo "bench $arm rc=$rc"; tail -1 gpurun_out/projlds_bench_$arm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['stage_ms_per_step'], d['config']['false_loop_closure_rejections'])"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
fi
