#!/bin/bash
# r03l: attention stage loop unrolled by 3 (constant ring slots) + one-statement row max: A/B vs ab_base
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" tests/test_lightglue_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03l_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03l_tests.log; [ $rc -eq 0 ] || exit $rc
for arm in new base new base; do
  if [ $arm = new ]; then timeout -k 10 200 python -u tools/attn_bench.py --pairs 1024 --len 2048 --iters 5 > gpurun_out/r03l_attn_$arm.json || exit 1
  else timeout -k 10 200 python -u tools/ab_run.py --lib-dir ab_base tools/attn_bench.py --pairs 1024 --len 2048 --iters 5 > gpurun_out/r03l_attn_$arm.json || exit 1; fi
  echo $arm $(cat gpurun_out/r03l_attn_$arm.json)
done
