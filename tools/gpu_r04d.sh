#!/bin/bash
# r04d: split-bf16 ViT -- parity tests, retrieval vs fp32 at bench scale, bench cost A/B
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_vit_gpu.py > gpurun_out/r04d_vit_tests.log 2>&1 || { tail -30 gpurun_out/r04d_vit_tests.log; exit 1; }
tail -3 gpurun_out/r04d_vit_tests.log
timeout -k 10 400 python -u tools/bench_parity.py retrieval --out gpurun_out/r04d_retrieval_split.npz > gpurun_out/r04d_retrieval.log 2>&1 || { tail -20 gpurun_out/r04d_retrieval.log; exit 1; }
tail -1 gpurun_out/r04d_retrieval.log
for v in bf16 split; do
  timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --loftr-pairs 0 --vit $v > gpurun_out/r04d_bench_$v.json 2> gpurun_out/r04d_bench_$v.err || { tail -5 gpurun_out/r04d_bench_$v.err; exit 1; }
  python3 -c "import json,sys; l=json.loads(open('gpurun_out/r04d_bench_$v.json').read().strip().splitlines()[-1]); r=l['roofline']; print('$v', l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections'], {k: v for k, v in r['stage_ms_per_step'].items() if k.startswith('vit')})"
done
