#!/bin/bash
# r04n: same-box A/B of the fused block tail built with / without SLP (ABAB, LightGlue stage
# bench), then the rocprof kernel-trace summary of a default bench run
set -u
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_vit_gpu.py tests/test_superpoint_gpu.py tests/test_kernels_gpu.py tests/test_loftr_gpu.py > gpurun_out/r04n_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r04n_pytest.log
[ $rc = 0 ] || exit $rc
for arm in ctl slpon ctl slpon; do
  timeout -k 10 240 python -u tools/ab_run.py --lib-dir ab_ffn_$arm tools/lg_bench.py --pairs 2048 --iters 2 >> gpurun_out/r04n_ab_$arm.log 2>&1 || { rc=$?; echo "$arm rc=$rc"; break; }
  echo "$arm $(grep '^{' gpurun_out/r04n_ab_$arm.log | tail -1 | head -c 400)"
done
[ $rc = 0 ] && { timeout -k 10 200 python -u tools/gemm_lib_probe.py > gpurun_out/r04n_gemm_lib.log 2>&1; rc=$?; tail -1 gpurun_out/r04n_gemm_lib.log; }
if [ $rc = 0 ]; then  # split-GEMM tile A/B (ABAB): 256 x 256 two-stage vs 192 x 192 three-stage
  for arm in tree s192 tree s192; do
    if [ $arm = tree ]; then timeout -k 10 200 python -u tools/vit_bench.py --vit split >> gpurun_out/r04n_vit_$arm.log 2>&1 || { rc=$?; break; }
    else timeout -k 10 200 python -u tools/ab_run.py --lib-dir ab_split192 tools/vit_bench.py --vit split >> gpurun_out/r04n_vit_$arm.log 2>&1 || { rc=$?; break; }; fi
    echo "$arm $(grep '^{' gpurun_out/r04n_vit_$arm.log | tail -1)"
  done
fi
[ $rc = 0 ] && timeout -k 10 700 bash tools/gpu_profile.sh r04n; rc2=$?
[ $rc = 0 ] && rc=$rc2
exit $rc
