#!/bin/bash
# r03aj: attention tile, MFMA shape (16x16x32 / 32x32x16) x V tile prefetch distance (1 / 2 stages),
# in-kernel clock builds, two rounds; then parity tests on the tree build (16x16x32, V 2 ahead)
set -u
mkdir -p gpurun_out
for r in 1 2; do
for arm in clk16v2 clk16v1 clk32v2 clk32v1; do
  timeout -k 10 180 python3 tools/ab_run.py --lib-dir ab_$arm tools/attn_bench.py --pairs 1024 --iters 5 --clock 3 > gpurun_out/r03aj_$arm$r.log 2>&1 || exit 1
  echo "$arm $(tail -1 gpurun_out/r03aj_$arm$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print([(k, d[k]['ms'], d[k]['tflops'], d[k]['clock_ghz'], d[k]['tflops_at_2.4'], round(d[k]['max_abs_err'],4)) for k in ('self','cross')])")"
done
done
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_lightglue_gpu.py tests/test_vit_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03aj_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r03aj_pytest.log; exit $rc
