#!/bin/bash
# r04f: GPU suite + the default bench line (split ViT, LoFTR gate sub-object, ingest, configs[0], CPU baseline)
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04f_pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r04f_pytest_gpu.log; grep -E "FAILED|ERROR" gpurun_out/r04f_pytest_gpu.log | head -10
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 480 python -u bench.py > gpurun_out/r04f_bench.json 2> gpurun_out/r04f_bench.err || { tail -8 gpurun_out/r04f_bench.err; exit 1; }
python3 - <<'PY'
import json
l = json.loads(open('gpurun_out/r04f_bench.json').read().strip().splitlines()[-1])
r = l['roofline']
print(l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections'], r['kernel'], r['frac'], r['avg_launch_us'])
print(r['stage_ms_per_step'])
for k in ('loftr', 'ingest', 'configs0', 'cpu_baseline'):
    print(k, json.dumps(l.get(k))[:600])
PY
