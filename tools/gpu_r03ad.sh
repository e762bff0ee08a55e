#!/bin/bash
# r03ad: attention Q loads / O stores non-temporal (ab_attnt) vs cached (tree); both with the non-temporal FFN rows
set -u
mkdir -p gpurun_out
for arm in tree attnt tree attnt; do
  if [ $arm = tree ]; then timeout -k 10 300 python -u tools/lg_bench.py --pairs 4096 --frames 1024 --iters 2 > gpurun_out/r03ad_$arm.json 2>/dev/null || exit 1
  else timeout -k 10 300 python -u tools/ab_run.py --lib-dir ab_$arm tools/lg_bench.py --pairs 4096 --frames 1024 --iters 2 > gpurun_out/r03ad_$arm.json 2>/dev/null || exit 1; fi
  echo $arm $(tail -1 gpurun_out/r03ad_$arm.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_call'], d['attention']['ms_per_call'], d['ffn_fused']['ms_per_call'], d['qkv_proj']['ms_per_call'], d['matches_mean'])")
done
