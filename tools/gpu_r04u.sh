#!/bin/bash
# r04u: assignment GEMM (k_asg_sim) operand prefetch depth 1 / 2 / 3 k-steps, LightGlue stage bench
set -u
mkdir -p gpurun_out
for arm in tree asg2 asg3 tree asg2 asg3; do
  if [ $arm = tree ]; then timeout -k 10 240 python -u tools/lg_bench.py --pairs 2048 --iters 2 >> gpurun_out/r04u_lg_$arm.log 2>&1 || exit 1
  else timeout -k 10 240 python -u tools/ab_run.py --lib-dir ab_$arm tools/lg_bench.py --pairs 2048 --iters 2 >> gpurun_out/r04u_lg_$arm.log 2>&1 || exit 1; fi
  echo "lg $arm $(grep '^{' gpurun_out/r04u_lg_$arm.log | tail -1 | cut -c1-200)"
done
