#!/bin/bash
# r04q: same-box ABAB of LightGlue on a high-priority stream (RANSAC side stream fills gaps)
set -u
mkdir -p gpurun_out
for p in 0 1 0 1; do
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --loftr-pairs 0 --no-ingest --lg-priority $p > gpurun_out/r04q_prio$p.json 2> gpurun_out/r04q_prio$p.err || { echo "prio $p failed"; tail -3 gpurun_out/r04q_prio$p.err; exit 1; }
  python3 -c "import json; l=json.loads(open('gpurun_out/r04q_prio$p.json').read().strip().splitlines()[-1]); r=l['roofline']; print('prio $p', l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections']['total'], r['stage_ms_per_step']['lightglue_attention'])"
done
