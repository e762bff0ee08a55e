#!/bin/bash
# r03p: ViT attention on the pipelined varlen tile -- kernel + ViT + SALAD tests first, then full suite, bench
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_vit_gpu.py tests/test_salad_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03p_vit.log 2>&1; rc=$?; tail -3 gpurun_out/r03p_vit.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r03p_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03p_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r03p_bench.json 2> gpurun_out/r03p_bench.err || { tail -5 gpurun_out/r03p_bench.err; exit 1; }
python3 -c "import json; l=json.loads(open('gpurun_out/r03p_bench.json').read().strip().splitlines()[-1]); print(l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections'], json.dumps(l['roofline']['stage_ms_per_step']), json.dumps(l['roofline']['stage_rate']), l['roofline']['frac'])"
