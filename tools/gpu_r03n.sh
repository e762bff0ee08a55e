#!/bin/bash
# r03n: attention unrolled + row max and lane-half swap in one asm statement: A/B vs ab_base (pre-unroll)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_lightglue_gpu.py tests/test_superglue_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03n_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03n_tests.log; [ $rc -eq 0 ] || exit $rc
for arm in new base new base; do
  if [ $arm = new ]; then timeout -k 10 200 python -u tools/attn_bench.py --pairs 1024 --len 2048 --iters 5 > gpurun_out/r03n_attn_$arm.json || exit 1
  else timeout -k 10 200 python -u tools/ab_run.py --lib-dir ab_base tools/attn_bench.py --pairs 1024 --len 2048 --iters 5 > gpurun_out/r03n_attn_$arm.json || exit 1; fi
  echo $arm $(cat gpurun_out/r03n_attn_$arm.json)
done
