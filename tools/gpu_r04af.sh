#!/bin/bash
# r04af: fc1 epilogue timing probes on the split ViT GEMM: tree vs no stores (4) vs no GELU (8)
set -u
mkdir -p gpurun_out
for arm in tree nost nogelu tree nost nogelu; do
  if [ $arm = tree ]; then pre=""; elif [ $arm = nost ]; then pre="tools/ab_run.py --lib-dir ab_epinost"; else pre="tools/ab_run.py --lib-dir ab_epinogelu"; fi
  timeout -k 10 120 python -u $pre tools/vit_bench.py --vit split --frames 492 --batch 246 --iters 3 > gpurun_out/r04af_$arm.log 2>&1 || { echo "$arm failed"; tail -5 gpurun_out/r04af_$arm.log; exit 1; }
  echo "vit $arm $(grep '^{' gpurun_out/r04af_$arm.log | tail -1 | cut -c1-260)"
done
