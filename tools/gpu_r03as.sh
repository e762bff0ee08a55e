#!/bin/bash
# r03as: LightGlue pairs per call (bench.py --lg-chunk 4096 default / 5120 / 6144), same box, alternated
set -u
mkdir -p gpurun_out
for r in 1 2; do
for c in 4096 5120 6144; do
  timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --loftr-pairs 0 --lg-chunk $c > gpurun_out/r03as_${c}_$r.log 2>&1 || { tail -3 gpurun_out/r03as_${c}_$r.log; exit 1; }
  echo "chunk $c $(tail -1 gpurun_out/r03as_${c}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['roofline']['stage_ms_per_step']; print(d['value'], d['ms_per_step'], d['roofline']['frac'], s['lightglue_attention'], s['lightglue_ffn_fused'], d['config']['false_loop_closure_rejections']['total'])")"
done
done
