#!/bin/bash
# r03at: bench default (5120 LightGlue pairs per call), rocprof stats, PMC traffic of one 5120-pair call
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/r03at_bench.json 2> gpurun_out/r03at_bench.err || { tail -5 gpurun_out/r03at_bench.err; exit 1; }
python3 -c "import json; l=json.loads(open('gpurun_out/r03at_bench.json').read().strip().splitlines()[-1]); print(l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections']['total'], l['roofline']['frac'], l['roofline']['avg_launch_us'], l['roofline']['flops_per_launch'])"
timeout -k 10 700 bash tools/gpu_profile.sh r03at || exit 1
PAIRS=5120 timeout -k 10 600 bash tools/pmc_traffic.sh
