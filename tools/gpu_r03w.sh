#!/bin/bash
# r03w: k_attention_varlen determinism across shapes (in-tree build)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/attn_det_probe.py multi-level-indoor-slam_amd/mlgate > gpurun_out/r03w_attn.json 2> gpurun_out/r03w_attn.err || { tail -5 gpurun_out/r03w_attn.err; exit 1; }
cat gpurun_out/r03w_attn.json
