#!/bin/bash
# r04g: bf16-ViT bench arm (same box as r04f is not guaranteed) + FFN SLP hazard probe arms
set -u
mkdir -p gpurun_out
for v in split bf16; do
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --loftr-pairs 0 --no-ingest --vit $v > gpurun_out/r04g_bench_$v.json 2> gpurun_out/r04g_bench_$v.err || { tail -5 gpurun_out/r04g_bench_$v.err; exit 1; }
  python3 -c "import json; l=json.loads(open('gpurun_out/r04g_bench_$v.json').read().strip().splitlines()[-1]); r=l['roofline']; print('$v', l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections']['total'], r['stage_ms_per_step'])"
done
for arm in ctl slp slpwait slpnont; do
  timeout -k 10 240 python -u tools/ab_run.py --lib-dir ab_ffn_$arm tools/ffn_interference.py --victims ffn --partners attn,proj --repeats 12 > gpurun_out/r04g_ffn_$arm.log 2>&1 || { tail -5 gpurun_out/r04g_ffn_$arm.log; exit 1; }
  echo "$arm $(tail -1 gpurun_out/r04g_ffn_$arm.log)"
done
