#!/bin/bash
# r03r: attention pad probe (ViT layout)
set -u
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/attn_pad_probe.py > gpurun_out/r03r_pad.json 2> gpurun_out/r03r_pad.err || { tail -5 gpurun_out/r03r_pad.err; exit 1; }
cat gpurun_out/r03r_pad.json
