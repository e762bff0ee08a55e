#!/bin/bash
# HISTORICAL (kept as the recipe of the profiles it produced): it switches arms through
# runtime knobs (MLG_FFN_* / MLG_PROJ_* / MLG_GEMM_VARIANT env vars, MLGATE_LIB_DIR) that the
# library no longer reads, so both arms would now run the same build.  Build each arm
# with -D flags instead and load it through tools/ab_run.py --lib-dir (tools/gpu_r03ag.sh).
echo "$0: historical recipe; its runtime A/B knobs are gone (see header)" >&2; exit 2
# Same-box A/B: FFN launch form (MLG_FFN_GRID 0 = one workgroup per tile, 2 = persistent)
# x projection tile (MLG_PROJ_MT 2 = 64 tokens, 4 = 128), then the kernel tests and a
# short bench with the defaults.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_lightglue_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ab_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for cfg in "0 4" "2 2" "0 2" "2 4" "0 4"; do
  set -- $cfg
  MLG_FFN_GRID=$1 MLG_PROJ_MT=$2 timeout -k 10 120 python3 tools/proj_ab.py --iters 10 > gpurun_out/ab_$1_$2.log 2>&1
  rc=$?; echo "ffn_grid=$1 proj_mt=$2 rc=$rc $(cat gpurun_out/ab_$1_$2.log | tail -1)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for cfg in "0 4" "2 2"; do
  set -- $cfg
  MLG_FFN_GRID=$1 MLG_PROJ_MT=$2 timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_bench_$1_$2.log 2>&1
  rc=$?; echo "bench ffn_grid=$1 proj_mt=$2 rc=$rc"; tail -1 gpurun_out/ab_bench_$1_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['stage_ms_per_step'])"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
