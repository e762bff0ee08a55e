#!/bin/bash
# r03v: attention prologue hazard pad; ViT attention on the pipelined tile -- determinism probes
# (kernel at ViT scale, ViT forward, LightGlue single / two streams / noise), full GPU suite, bench
set -u
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/attn_det_probe.py multi-level-indoor-slam_amd/mlgate 123 > gpurun_out/r03v_attn.json 2> gpurun_out/r03v_attn.err || { tail -5 gpurun_out/r03v_attn.err; exit 1; }
cat gpurun_out/r03v_attn.json
timeout -k 10 300 python -u tools/vit_det.py > gpurun_out/r03v_vitdet.json 2> gpurun_out/r03v_vitdet.err || { tail -5 gpurun_out/r03v_vitdet.err; exit 1; }
cat gpurun_out/r03v_vitdet.json
timeout -k 10 400 python -u tools/lg_determinism.py --modes single,threads2,noise > gpurun_out/r03v_lgdet.log 2>&1 || { tail -5 gpurun_out/r03v_lgdet.log; exit 1; }
grep summary gpurun_out/r03v_lgdet.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r03v_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03v_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r03v_bench.json 2> gpurun_out/r03v_bench.err || { tail -5 gpurun_out/r03v_bench.err; exit 1; }
python3 -c "import json; l=json.loads(open('gpurun_out/r03v_bench.json').read().strip().splitlines()[-1]); print(l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections'], json.dumps(l['roofline']['stage_ms_per_step']), json.dumps(l['roofline']['stage_rate']), l['roofline']['frac'])"
