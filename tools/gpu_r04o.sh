#!/bin/bash
# r04o: LightGlue remainder chunk split (shorter RANSAC tail); whole GPU suite + default bench
set -u
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 700 $T -m gpu tests > gpurun_out/r04o_pytest_gpu.log 2>&1 && echo "suite ok" &&
timeout -k 10 400 python -u bench.py > gpurun_out/r04o_bench.json 2> gpurun_out/r04o_bench.err && echo "bench ok"
rc=$?
echo "rc=$rc"
tail -2 gpurun_out/r04o_pytest_gpu.log
python3 -c "import json; l=json.loads(open('gpurun_out/r04o_bench.json').read().strip().splitlines()[-1]); r=l['roofline']; print(l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections']['total'], r['frac'], r['stage_ms_per_step'])" 2>/dev/null
exit $rc
