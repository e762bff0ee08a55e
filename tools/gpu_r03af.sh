#!/bin/bash
# HISTORICAL (kept as the recipe of the profiles it produced): it switches arms through
# runtime knobs (MLG_FFN_* / MLG_PROJ_* / MLG_GEMM_VARIANT env vars, MLGATE_LIB_DIR) that the
# library no longer reads, so both arms would now run the same build.  Build each arm
# with -D flags instead and load it through tools/ab_run.py --lib-dir (tools/gpu_r03ag.sh).
echo "$0: historical recipe; its runtime A/B knobs are gone (see header)" >&2; exit 2
# r03af: fused FFN on 8 waves per 64-row tile (MLG_FFN_WAVES=8, 4 waves / SIMD, 128 VGPRs) vs 4 waves (default)
set -u
mkdir -p gpurun_out
MLG_FFN_WAVES=8 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "lg_ffn" -x -q --timeout 200 --timeout-method thread > gpurun_out/r03af_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r03af_tests.log; [ $rc -eq 0 ] || exit $rc
for arm in w4 w8 w4 w8; do
  if [ $arm = w8 ]; then export MLG_FFN_WAVES=8; else unset MLG_FFN_WAVES; fi
  timeout -k 10 300 python -u tools/lg_bench.py --pairs 4096 --frames 1024 --iters 2 > gpurun_out/r03af_$arm.json 2>/dev/null || exit 1
  echo $arm $(tail -1 gpurun_out/r03af_$arm.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_call'], d['ffn_fused']['ms_per_call'], d['matches_mean'])")
done
