#!/bin/bash
# r03z: row max compiler-visible (no IEEE canonicalisation, hipcc pads the MFMA reads) vs the padded asm
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/attn_det_probe.py ab_cxx > gpurun_out/r03z_attn_cxx.json 2> gpurun_out/r03z_attn_cxx.err || { tail -5 gpurun_out/r03z_attn_cxx.err; exit 1; }
echo cxx $(cat gpurun_out/r03z_attn_cxx.json)
for arm in tree cxx tree cxx tree cxx; do
  if [ $arm = tree ]; then timeout -k 10 200 python -u tools/attn_bench.py --pairs 1024 --len 2048 --iters 5 > gpurun_out/r03z_t_$arm.json || exit 1
  else timeout -k 10 200 python -u tools/ab_run.py --lib-dir ab_$arm tools/attn_bench.py --pairs 1024 --len 2048 --iters 5 > gpurun_out/r03z_t_$arm.json || exit 1; fi
  echo $arm $(cat gpurun_out/r03z_t_$arm.json)
done
