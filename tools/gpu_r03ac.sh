#!/bin/bash
# r03ac: FFN tile rows / residual through non-temporal accesses (ab_nt) vs cached (tree)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_run.py --lib-dir ab_nt -m pytest tests/test_kernels_gpu.py -k "lg_ffn" -x -q > gpurun_out/r03ac_tests.log 2>&1 || true
tail -1 gpurun_out/r03ac_tests.log
for arm in tree nt tree nt; do
  if [ $arm = tree ]; then timeout -k 10 300 python -u tools/lg_bench.py --pairs 4096 --frames 1024 --iters 2 > gpurun_out/r03ac_$arm.json 2>/dev/null || exit 1
  else timeout -k 10 300 python -u tools/ab_run.py --lib-dir ab_$arm tools/lg_bench.py --pairs 4096 --frames 1024 --iters 2 > gpurun_out/r03ac_$arm.json 2>/dev/null || exit 1; fi
  echo $arm $(tail -1 gpurun_out/r03ac_$arm.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_call'], d['ffn_fused'], d['matches_mean'])")
done
