#!/bin/bash
# r03s: ViT determinism probe on HEAD's libraries (ab_base) vs the working tree
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_run.py --lib-dir ab_base tools/vit_det.py > gpurun_out/r03s_vitdet_base.json 2> gpurun_out/r03s_base.err || { tail -5 gpurun_out/r03s_base.err; exit 1; }
echo base $(cat gpurun_out/r03s_vitdet_base.json)
timeout -k 10 300 python -u tools/vit_det.py > gpurun_out/r03s_vitdet_new.json 2> gpurun_out/r03s_new.err || { tail -5 gpurun_out/r03s_new.err; exit 1; }
echo new $(cat gpurun_out/r03s_vitdet_new.json)
