#!/bin/bash
# r04p: same-box ABAB of the LightGlue tail-chunk split (--lg-tail 0 vs 4) on the bench
set -u
mkdir -p gpurun_out
for t in 0 4 0 4; do
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --loftr-pairs 0 --no-ingest --lg-tail $t > gpurun_out/r04p_tail$t.json 2> gpurun_out/r04p_tail$t.err || { echo "tail $t failed"; tail -3 gpurun_out/r04p_tail$t.err; exit 1; }
  python3 -c "import json; l=json.loads(open('gpurun_out/r04p_tail$t.json').read().strip().splitlines()[-1]); r=l['roofline']; print('tail $t', l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections']['total'], r['stage_ms_per_step']['lightglue_attention'])"
done
