#!/bin/bash
# r03aw: ViT frames per batch on the bench (--batch 123 default / 246), same box, alternated
set -u
mkdir -p gpurun_out
for r in 1 2; do
for b in 123 246; do
  timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --loftr-pairs 0 --batch $b > gpurun_out/r03aw_${b}_$r.log 2>&1 || { tail -3 gpurun_out/r03aw_${b}_$r.log; exit 1; }
  echo "batch $b $(tail -1 gpurun_out/r03aw_${b}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['roofline']['stage_ms_per_step']; print(d['value'], d['ms_per_step'], round(sum(v for k,v in s.items() if k.startswith('vit')),1), d['config']['false_loop_closure_rejections']['total'])")"
done
done
