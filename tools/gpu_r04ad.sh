#!/bin/bash
# r04ad: split ViT GEMM (k_gemm256s) timing probes: tree vs no K-loop DMA (1), no epilogue
# (2), neither (3) -- results of the probe arms are wrong by design; times only
set -u
mkdir -p gpurun_out
for arm in tree nodma noepi none tree nodma noepi none; do
  if [ $arm = tree ]; then pre=""; else pre="tools/ab_run.py --lib-dir ab_s256$arm"; fi
  timeout -k 10 120 python -u $pre tools/vit_bench.py --vit split --frames 492 --batch 246 --iters 3 > gpurun_out/r04ad_$arm.log 2>&1 || { echo "$arm failed"; tail -5 gpurun_out/r04ad_$arm.log; exit 1; }
  echo "vit $arm $(grep '^{' gpurun_out/r04ad_$arm.log | tail -1)"
done
