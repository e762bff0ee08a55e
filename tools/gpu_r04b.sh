#!/bin/bash
# r04b: ViT precision sites probe + SuperPoint oracle timing on a steady shape
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/vit_precision_probe.py > gpurun_out/r04b_vitprec.log 2>&1 || { tail -20 gpurun_out/r04b_vitprec.log; exit 1; }
cat gpurun_out/r04b_vitprec.log
timeout -k 10 300 python -u tools/bench_parity.py probe > gpurun_out/r04b_probe.log 2>&1 || { tail -20 gpurun_out/r04b_probe.log; exit 1; }
tail -3 gpurun_out/r04b_probe.log
