#!/bin/bash
# r03ax: final bench default (246 ViT frames per batch, 5120 LightGlue pairs per call) + rocprof stats
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ax_smoke.log 2>&1 || { tail -5 gpurun_out/r03ax_smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/r03ax_bench.json 2> gpurun_out/r03ax_bench.err || { tail -5 gpurun_out/r03ax_bench.err; exit 1; }
python3 -c "import json; l=json.loads(open('gpurun_out/r03ax_bench.json').read().strip().splitlines()[-1]); r=l['roofline']; print(l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections']['total'], r['frac'], r['avg_launch_us'], r['traffic'], l['cpu_baseline']['value'])"
timeout -k 10 700 bash tools/gpu_profile.sh r03ax
