#!/bin/bash
# r03am: in-kernel clocks of the LightGlue kernels (attention, fused FFN, projections) during
# back-to-back 4096-pair LightGlue calls (tools/clock_probe_build.py library ab_clkall), twice
set -u
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python3 tools/ab_run.py --lib-dir ab_clkall tools/lg_bench.py --pairs 4096 --frames 1024 --iters 2 --clock 5 > gpurun_out/r03am_$r.json 2> gpurun_out/r03am_$r.err || { tail -5 gpurun_out/r03am_$r.err; exit 1; }
  tail -1 gpurun_out/r03am_$r.json
done
