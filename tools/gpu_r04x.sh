#!/bin/bash
# r04x: LightGlue init with the layer-0 row gather folded in (tree) vs the separate gather pass
# (ab_gather, -DMLG_LG_INIT_FUSED=0): LightGlue GPU tests, then same-box ABAB of the bench
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lightglue_gpu.py > gpurun_out/r04x_lg_tests.log 2>&1 || { echo "lg tests failed"; tail -20 gpurun_out/r04x_lg_tests.log; exit 1; }
tail -1 gpurun_out/r04x_lg_tests.log
for arm in tree gather tree gather; do
  if [ $arm = tree ]; then cmd="python -u bench.py"; else cmd="python -u tools/ab_run.py --lib-dir ab_gather bench.py"; fi
  timeout -k 10 300 $cmd --steps 2 --warmup 1 --no-cpu-baseline --loftr-pairs 0 --no-ingest > gpurun_out/r04x_$arm.json 2> gpurun_out/r04x_$arm.err || { echo "$arm failed"; tail -3 gpurun_out/r04x_$arm.err; exit 1; }
  python3 -c "import json; l=json.loads(open('gpurun_out/r04x_$arm.json').read().strip().splitlines()[-1]); r=l['roofline']; print('$arm', l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections']['total'], l['config']['pairs_geometrically_valid'], r['stage_ms_per_step']['lightglue_attention'])"
done
