#!/bin/bash
# r03ai: attention tile on v_mfma_f32_16x16x32_bf16 (tree) vs the 32x32x16 form (ab_a32):
# parity tests on the tree build, then in-kernel clock builds (ab_clk16 / ab_clk) and bench.py
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_lightglue_gpu.py tests/test_vit_gpu.py tests/test_salad_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03ai_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03ai_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for arm in clk16 clk; do
  timeout -k 10 180 python3 tools/ab_run.py --lib-dir ab_$arm tools/attn_bench.py --pairs 1024 --iters 5 --clock 3 > gpurun_out/r03ai_$arm$r.log 2>&1 || exit 1
  echo "$arm $(tail -1 gpurun_out/r03ai_$arm$r.log)"
done
done
for arm in tree a32; do
  if [ $arm = tree ]; then timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03ai_bench_$arm.log 2>&1 || exit 1
  else timeout -k 10 400 python3 tools/ab_run.py --lib-dir ab_$arm bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03ai_bench_$arm.log 2>&1 || exit 1; fi
  echo "bench $arm"; tail -1 gpurun_out/r03ai_bench_$arm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['stage_ms_per_step'], d['config']['false_loop_closure_rejections']['total'])"
done
