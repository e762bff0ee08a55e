#!/bin/bash
# r03x: attention determinism with the MFMA->asm wait states: pad in the last stage only (tree) vs before every
# block max (ab_nopall); attention timing of both and of HEAD (ab_base)
set -u
mkdir -p gpurun_out
for arm in tree nopall; do
  d=multi-level-indoor-slam_amd/mlgate; [ $arm = nopall ] && d=ab_nopall
  timeout -k 10 300 python -u tools/attn_det_probe.py $d > gpurun_out/r03x_attn_$arm.json 2> gpurun_out/r03x_attn_$arm.err || { tail -5 gpurun_out/r03x_attn_$arm.err; exit 1; }
  echo $arm $(cat gpurun_out/r03x_attn_$arm.json)
done
for arm in tree nopall base tree nopall base; do
  if [ $arm = tree ]; then timeout -k 10 200 python -u tools/attn_bench.py --pairs 1024 --len 2048 --iters 5 > gpurun_out/r03x_t_$arm.json || exit 1
  else timeout -k 10 200 python -u tools/ab_run.py --lib-dir ab_$arm tools/attn_bench.py --pairs 1024 --len 2048 --iters 5 > gpurun_out/r03x_t_$arm.json || exit 1; fi
  echo $arm $(cat gpurun_out/r03x_t_$arm.json)
done
