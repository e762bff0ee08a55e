#!/bin/bash
# r03u: is k_attention_varlen deterministic at ViT scale (ab_vit build)?  And the ViT forward again.
set -u
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/attn_det_probe.py ab_vit 123 > gpurun_out/r03u_attn.json 2> gpurun_out/r03u_attn.err || { tail -5 gpurun_out/r03u_attn.err; exit 1; }
cat gpurun_out/r03u_attn.json
timeout -k 10 300 python -u tools/ab_run.py --lib-dir ab_vit tools/vit_det.py > gpurun_out/r03u_vitdet.json 2> gpurun_out/r03u_vitdet.err || { tail -5 gpurun_out/r03u_vitdet.err; exit 1; }
cat gpurun_out/r03u_vitdet.json
