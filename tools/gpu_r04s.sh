#!/bin/bash
# r04s: LightGlue attention 4 vs 8 waves per workgroup (ABAB, LightGlue stage bench); then the
# whole GPU suite and the default bench with the 8-wave split ViT attention
set -u
mkdir -p gpurun_out
for arm in tree lg8 tree lg8; do
  if [ $arm = tree ]; then timeout -k 10 240 python -u tools/lg_bench.py --pairs 2048 --iters 2 >> gpurun_out/r04s_lg_$arm.log 2>&1 || exit 1
  else timeout -k 10 240 python -u tools/ab_run.py --lib-dir ab_lg8 tools/lg_bench.py --pairs 2048 --iters 2 >> gpurun_out/r04s_lg_$arm.log 2>&1 || exit 1; fi
  echo "lg $arm $(grep '^{' gpurun_out/r04s_lg_$arm.log | tail -1 | cut -c1-330)"
done
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 700 $T -m gpu tests > gpurun_out/r04s_pytest_gpu.log 2>&1 && echo "suite ok" &&
timeout -k 10 400 python -u bench.py > gpurun_out/r04s_bench.json 2> gpurun_out/r04s_bench.err && echo "bench ok"
rc=$?
echo "rc=$rc"; tail -2 gpurun_out/r04s_pytest_gpu.log
python3 -c "import json; l=json.loads(open('gpurun_out/r04s_bench.json').read().strip().splitlines()[-1]); r=l['roofline']; print(l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections']['total'], r['frac'], r['stage_ms_per_step'])" 2>/dev/null
exit $rc
