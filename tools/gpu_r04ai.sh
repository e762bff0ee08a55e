#!/bin/bash
# r04ai: evidence run -- whole GPU suite, smoke(), default bench, rocprof of a bench run
set -u
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 700 $T -m gpu tests > gpurun_out/r04ai_pytest_gpu.log 2>&1 && echo "suite ok" &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04ai_smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 400 python -u bench.py > gpurun_out/r04ai_bench.json 2> gpurun_out/r04ai_bench.err && echo "bench ok" &&
timeout -k 10 600 bash tools/gpu_profile.sh r04ai > gpurun_out/r04ai_prof.log 2>&1 && echo "prof ok"
rc=$?
echo "rc=$rc"; tail -2 gpurun_out/r04ai_pytest_gpu.log; tail -2 gpurun_out/r04ai_smoke.log
python3 -c "import json; l=json.loads(open('gpurun_out/r04ai_bench.json').read().strip().splitlines()[-1]); r=l['roofline']; print(l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections']['total'], r['frac'], r['traffic'], r['stage_ms_per_step'])" 2>/dev/null
exit $rc
