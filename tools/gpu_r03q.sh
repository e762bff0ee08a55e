#!/bin/bash
# r03q: ViT determinism probe (batch / position / concurrency); RANSAC two-round tests; bench
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/vit_det.py > gpurun_out/r03q_vitdet.json 2> gpurun_out/r03q_vitdet.err || { tail -5 gpurun_out/r03q_vitdet.err; exit 1; }
cat gpurun_out/r03q_vitdet.json
timeout -k 10 600 python -u -m pytest tests/test_ransac_gpu.py tests/test_pipeline_gpu.py tests/test_verify_gpu.py tests/test_decisions_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r03q_ransac.log 2>&1; rc=$?; tail -3 gpurun_out/r03q_ransac.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline --loftr-pairs 0 > gpurun_out/r03q_bench.json 2> gpurun_out/r03q_bench.err || { tail -5 gpurun_out/r03q_bench.err; exit 1; }
python3 -c "import json; l=json.loads(open('gpurun_out/r03q_bench.json').read().strip().splitlines()[-1]); print(l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections'], json.dumps(l['roofline']['stage_ms_per_step']), json.dumps(l['roofline']['stage_rate']), l['roofline']['frac'])"
