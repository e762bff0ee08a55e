#!/bin/bash
# r03ah: in-kernel clock of the attention tile (tools/clock_probe_build.py builds) under
# 3 s of back-to-back launches on random data: HEAD tile (ab_clk) and the no-exp timing probe (ab_clkp2)
set -u
mkdir -p gpurun_out
for arm in clk clkp2 clk clkp2; do
  timeout -k 10 180 python3 tools/ab_run.py --lib-dir ab_$arm tools/attn_bench.py --pairs 1024 --iters 5 --clock 3 > gpurun_out/r03ah_$arm.log 2>&1 || exit 1
  echo "$arm $(tail -1 gpurun_out/r03ah_$arm.log)"
done
