#!/bin/bash
# r03aq: attention tile, waves whose 64 queries all lie past the task's end skip the
# compute and only stage K / V (tree) vs HEAD (ab_head): parity tests on the tree, then
# lg_bench (bench-shaped 4096-pair calls, pruning on) and attn_bench ragged, arms alternated, then bench.py
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_lightglue_gpu.py tests/test_vit_gpu.py tests/test_salad_gpu.py tests/test_superglue_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03aq_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/r03aq_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for arm in tree head; do
  if [ $arm = tree ]; then P=""; else P="tools/ab_run.py --lib-dir ab_head"; fi
  timeout -k 10 300 python3 $P tools/lg_bench.py --pairs 4096 --frames 1024 --iters 2 > gpurun_out/r03aq_lg_$arm$r.json 2>/dev/null || exit 1
  timeout -k 10 120 python3 $P tools/attn_bench.py --pairs 1024 --iters 5 --ragged > gpurun_out/r03aq_at_$arm$r.json 2>/dev/null || exit 1
  echo "$arm lg $(tail -1 gpurun_out/r03aq_lg_$arm$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_call'], d['attention'], d['matches_mean'])") ragged $(tail -1 gpurun_out/r03aq_at_$arm$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['self']['ms'], d['cross']['ms'], round(d['self']['max_abs_err'],4))")"
done
done
for arm in tree head; do
  if [ $arm = tree ]; then P=""; else P="tools/ab_run.py --lib-dir ab_head"; fi
  timeout -k 10 400 python3 $P bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03aq_bench_$arm.log 2>&1 || exit 1
  echo "bench $arm"; tail -1 gpurun_out/r03aq_bench_$arm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['roofline']['stage_ms_per_step']; print(d['value'], d['ms_per_step'], d['roofline']['frac'], s['lightglue_attention'], s['vit_attention'], d['config']['false_loop_closure_rejections']['total'])"
done
