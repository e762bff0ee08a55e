#!/bin/bash
# r04ac: LightGlue attention with the optimistic softmax (tree) vs the max-first lazy
# rescale (ab_attnmax, -DMLG_ATTN_OPT=0): kernel + LightGlue tests, determinism probe,
# attention microbench (ABAB, with max error vs f32 torch), LightGlue stage bench (ABAB),
# then bench.py ABAB
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_lightglue_gpu.py > gpurun_out/r04ac_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r04ac_tests.log; exit 1; }
tail -1 gpurun_out/r04ac_tests.log
timeout -k 10 200 python -u tools/attn_det_probe.py multi-level-indoor-slam_amd/mlgate > gpurun_out/r04ac_det.log 2>&1 || { echo "det failed"; tail -5 gpurun_out/r04ac_det.log; exit 1; }
echo "det $(tail -1 gpurun_out/r04ac_det.log)"
for arm in tree max tree max; do
  if [ $arm = tree ]; then pre=""; else pre="tools/ab_run.py --lib-dir ab_attnmax"; fi
  timeout -k 10 120 python -u $pre tools/attn_bench.py --pairs 256 > gpurun_out/r04ac_attn_$arm.log 2>&1 || { echo "attn $arm failed"; tail -5 gpurun_out/r04ac_attn_$arm.log; exit 1; }
  echo "attn $arm $(grep '^{' gpurun_out/r04ac_attn_$arm.log | tail -1)"
done
for arm in tree max tree max; do
  if [ $arm = tree ]; then pre=""; else pre="tools/ab_run.py --lib-dir ab_attnmax"; fi
  timeout -k 10 240 python -u $pre tools/lg_bench.py --pairs 2048 --iters 2 >> gpurun_out/r04ac_lg_$arm.log 2>&1 || { echo "lg $arm failed"; tail -5 gpurun_out/r04ac_lg_$arm.log; exit 1; }
  echo "lg $arm $(grep '^{' gpurun_out/r04ac_lg_$arm.log | tail -1 | cut -c1-420)"
done
for arm in tree max; do
  if [ $arm = tree ]; then cmd="python -u bench.py"; else cmd="python -u tools/ab_run.py --lib-dir ab_attnmax bench.py"; fi
  timeout -k 10 300 $cmd --steps 2 --warmup 1 --no-cpu-baseline --loftr-pairs 0 --no-ingest > gpurun_out/r04ac_b_$arm.json 2> gpurun_out/r04ac_b_$arm.err || { echo "bench $arm failed"; tail -3 gpurun_out/r04ac_b_$arm.err; exit 1; }
  python3 -c "import json; l=json.loads(open('gpurun_out/r04ac_b_$arm.json').read().strip().splitlines()[-1]); r=l['roofline']; print('bench $arm', l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections'], l['config']['pairs_geometrically_valid'], r['frac'], r['stage_ms_per_step']['lightglue_attention'])"
done
