#!/bin/bash
# r04ah: V^T waves of the split qkv GEMM staged transposed through LDS (tree) vs HEAD
# (ab_gemmold): ViT / kernel tests, tools/vit_bench.py ABAB (descriptor sha1 must match),
# bench.py ABAB
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_vit_gpu.py > gpurun_out/r04ah_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r04ah_tests.log; exit 1; }
tail -1 gpurun_out/r04ah_tests.log
for arm in tree old tree old; do
  if [ $arm = tree ]; then pre=""; else pre="tools/ab_run.py --lib-dir ab_gemmold"; fi
  timeout -k 10 120 python -u $pre tools/vit_bench.py --vit split --frames 492 --batch 246 --iters 3 > gpurun_out/r04ah_vit_$arm.log 2>&1 || { echo "vit $arm failed"; tail -5 gpurun_out/r04ah_vit_$arm.log; exit 1; }
  echo "vit $arm $(grep '^{' gpurun_out/r04ah_vit_$arm.log | tail -1)"
done
for arm in tree old; do
  if [ $arm = tree ]; then cmd="python -u bench.py"; else cmd="python -u tools/ab_run.py --lib-dir ab_gemmold bench.py"; fi
  timeout -k 10 300 $cmd --steps 2 --warmup 1 --no-cpu-baseline --loftr-pairs 0 --no-ingest > gpurun_out/r04ah_b_$arm.json 2> gpurun_out/r04ah_b_$arm.err || { echo "bench $arm failed"; tail -3 gpurun_out/r04ah_b_$arm.err; exit 1; }
  python3 -c "import json; l=json.loads(open('gpurun_out/r04ah_b_$arm.json').read().strip().splitlines()[-1]); r=l['roofline']; s=r['stage_ms_per_step']; print('bench $arm', l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections']['total'], l['config']['pairs_geometrically_valid'], {k: s[k] for k in s if k.startswith('vit')})"
done
