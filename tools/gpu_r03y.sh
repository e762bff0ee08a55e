#!/bin/bash
# r03y: attention with the MFMA->asm wait states before every block max; ViT on the pipelined tile:
# determinism probes, full GPU suite, smoke, bench, rocprof
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/attn_det_probe.py multi-level-indoor-slam_amd/mlgate > gpurun_out/r03y_attn.json 2> gpurun_out/r03y_attn.err || { tail -5 gpurun_out/r03y_attn.err; exit 1; }
cat gpurun_out/r03y_attn.json
timeout -k 10 300 python -u tools/vit_det.py > gpurun_out/r03y_vitdet.json 2> gpurun_out/r03y_vitdet.err || { tail -5 gpurun_out/r03y_vitdet.err; exit 1; }
cat gpurun_out/r03y_vitdet.json
timeout -k 10 400 python -u tools/lg_determinism.py --modes single,threads2,noise > gpurun_out/r03y_lgdet.log 2>&1 || { tail -5 gpurun_out/r03y_lgdet.log; exit 1; }
grep summary gpurun_out/r03y_lgdet.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r03y_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03y_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03y_smoke.log 2>&1 || { tail -5 gpurun_out/r03y_smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/r03y_bench.json 2> gpurun_out/r03y_bench.err || { tail -5 gpurun_out/r03y_bench.err; exit 1; }
python3 -c "import json; l=json.loads(open('gpurun_out/r03y_bench.json').read().strip().splitlines()[-1]); print(l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections'], json.dumps(l['roofline']['stage_ms_per_step']), json.dumps(l['roofline']['stage_rate']), l['roofline']['frac'])"
timeout -k 10 700 bash tools/gpu_profile.sh r03y
