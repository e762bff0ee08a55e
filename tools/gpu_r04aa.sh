#!/bin/bash
# r04aa: FFN with ReLU as a template argument (tree: one straight-line GELU epilogue) vs the
# run-time flag (ab_ffnold: HEAD's lg_ffn.hip): kernel tests, output hashes + ms (ABAB),
# co-scheduling interference probe on the tree build, LightGlue stage bench (ABAB)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "ffn or deterministic" > gpurun_out/r04aa_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r04aa_tests.log; exit 1; }
tail -1 gpurun_out/r04aa_tests.log
for arm in tree old tree old; do
  if [ $arm = tree ]; then pre=""; else pre="tools/ab_run.py --lib-dir ab_ffnold"; fi
  timeout -k 10 120 python -u $pre tools/proj_pipe_check.py > gpurun_out/r04aa_chk_$arm.log 2>&1 || { echo "check $arm failed"; tail -5 gpurun_out/r04aa_chk_$arm.log; exit 1; }
  echo "chk $arm $(tail -1 gpurun_out/r04aa_chk_$arm.log)"
done
timeout -k 10 300 python -u tools/ffn_interference.py > gpurun_out/r04aa_interference.log 2>&1 || { echo "interference failed"; tail -5 gpurun_out/r04aa_interference.log; exit 1; }
tail -12 gpurun_out/r04aa_interference.log
for arm in tree old tree old; do
  if [ $arm = tree ]; then pre=""; else pre="tools/ab_run.py --lib-dir ab_ffnold"; fi
  timeout -k 10 240 python -u $pre tools/lg_bench.py --pairs 2048 --iters 2 >> gpurun_out/r04aa_lg_$arm.log 2>&1 || { echo "lg $arm failed"; tail -5 gpurun_out/r04aa_lg_$arm.log; exit 1; }
  echo "lg $arm $(grep '^{' gpurun_out/r04aa_lg_$arm.log | tail -1 | cut -c1-420)"
done
