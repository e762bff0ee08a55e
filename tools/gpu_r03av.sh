#!/bin/bash
# r03av: SuperPoint frames per batch on the bench (--sp-batch 64 default / 128 / 256), same box, alternated
set -u
mkdir -p gpurun_out
for r in 1 2; do
for b in 64 128 256; do
  timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --loftr-pairs 0 --sp-batch $b > gpurun_out/r03av_${b}_$r.log 2>&1 || { tail -3 gpurun_out/r03av_${b}_$r.log; exit 1; }
  echo "sp-batch $b $(tail -1 gpurun_out/r03av_${b}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['roofline']['stage_ms_per_step']; print(d['value'], d['ms_per_step'], s['superpoint_conv3x3'], d['config']['false_loop_closure_rejections']['total'])")"
done
done
