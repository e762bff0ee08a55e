#!/bin/bash
# r04z: pipelined resident projections (tree: epilogue of tile t-1 inside tile t's GEMM) vs
# the serial resident form (ab_projres, -DMLG_PROJ_PIPE=0): kernel tests, output hashes +
# ms per launch (ABAB), then the LightGlue stage bench (ABAB)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "lg_proj or deterministic" > gpurun_out/r04z_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r04z_tests.log; exit 1; }
tail -1 gpurun_out/r04z_tests.log
for arm in tree res tree res; do
  if [ $arm = tree ]; then pre=""; else pre="tools/ab_run.py --lib-dir ab_projres"; fi
  timeout -k 10 120 python -u $pre tools/proj_pipe_check.py > gpurun_out/r04z_chk_$arm.log 2>&1 || { echo "check $arm failed"; tail -5 gpurun_out/r04z_chk_$arm.log; exit 1; }
  echo "chk $arm $(tail -1 gpurun_out/r04z_chk_$arm.log)"
done
for arm in tree res tree res; do
  if [ $arm = tree ]; then pre=""; else pre="tools/ab_run.py --lib-dir ab_projres"; fi
  timeout -k 10 240 python -u $pre tools/lg_bench.py --pairs 2048 --iters 2 >> gpurun_out/r04z_lg_$arm.log 2>&1 || { echo "lg $arm failed"; tail -5 gpurun_out/r04z_lg_$arm.log; exit 1; }
  echo "lg $arm $(grep '^{' gpurun_out/r04z_lg_$arm.log | tail -1 | cut -c1-420)"
done
