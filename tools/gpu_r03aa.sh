#!/bin/bash
# r03aa: attention run-to-run regression test; FFN residual prefetch before the ffn2 GEMM (tree) vs loaded after it (ab_xrlate)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "run_to_run or lg_ffn" -x -q --timeout 200 --timeout-method thread > gpurun_out/r03aa_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03aa_tests.log; [ $rc -eq 0 ] || exit $rc
for arm in tree xrlate tree xrlate; do
  if [ $arm = tree ]; then timeout -k 10 300 python -u tools/lg_bench.py --pairs 4096 --frames 1024 --iters 2 > gpurun_out/r03aa_$arm.json 2>/dev/null || exit 1
  else timeout -k 10 300 python -u tools/ab_run.py --lib-dir ab_$arm tools/lg_bench.py --pairs 4096 --frames 1024 --iters 2 > gpurun_out/r03aa_$arm.json 2>/dev/null || exit 1; fi
  echo $arm $(tail -1 gpurun_out/r03aa_$arm.json | cut -c1-600)
done
