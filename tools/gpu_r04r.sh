#!/bin/bash
# r04r: 8-wave split ViT attention (two waves per SIMD) -- tests, ViT A/B against the 4-wave
# build (ab_ffn_ctl), LightGlue stage A/B (its tile's code path was re-templated), and the
# LightGlue stream-priority bench A/B
set -u
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_vit_gpu.py tests/test_kernels_gpu.py tests/test_lightglue_gpu.py > gpurun_out/r04r_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r04r_pytest.log
[ $rc = 0 ] || exit $rc
for arm in tree old tree old; do
  if [ $arm = tree ]; then timeout -k 10 200 python -u tools/vit_bench.py --vit split >> gpurun_out/r04r_vit_$arm.log 2>&1 || exit 1
  else timeout -k 10 200 python -u tools/ab_run.py --lib-dir ab_ffn_ctl tools/vit_bench.py --vit split >> gpurun_out/r04r_vit_$arm.log 2>&1 || exit 1; fi
  echo "vit $arm $(grep '^{' gpurun_out/r04r_vit_$arm.log | tail -1 | cut -c1-330)"
done
for arm in tree old; do
  if [ $arm = tree ]; then timeout -k 10 240 python -u tools/lg_bench.py --pairs 2048 --iters 2 >> gpurun_out/r04r_lg_$arm.log 2>&1 || exit 1
  else timeout -k 10 240 python -u tools/ab_run.py --lib-dir ab_ffn_ctl tools/lg_bench.py --pairs 2048 --iters 2 >> gpurun_out/r04r_lg_$arm.log 2>&1 || exit 1; fi
  echo "lg $arm $(grep '^{' gpurun_out/r04r_lg_$arm.log | tail -1 | cut -c1-330)"
done
for p in 0 1; do
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --loftr-pairs 0 --no-ingest --lg-priority $p > gpurun_out/r04r_prio$p.json 2> gpurun_out/r04r_prio$p.err || { echo "prio $p failed"; tail -3 gpurun_out/r04r_prio$p.err; exit 1; }
  python3 -c "import json; l=json.loads(open('gpurun_out/r04r_prio$p.json').read().strip().splitlines()[-1]); r=l['roofline']; print('prio $p', l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections']['total'], r['stage_ms_per_step'])"
done
