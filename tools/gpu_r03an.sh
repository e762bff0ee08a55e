#!/bin/bash
# r03an(b): fused FFN weight-ring depth: msg / ffn2 phases RING1 2 (r12), ffn1 RING2 2 / 8 (r22, r28) vs 4 / 4 (tree),
# tools/lg_bench.py 4096-pair calls, arms alternated twice (results must be identical: same MFMA order)
set -u
mkdir -p gpurun_out
for r in 1 2; do
for arm in tree r12 r22 r28; do
  if [ $arm = tree ]; then timeout -k 10 300 python3 tools/lg_bench.py --pairs 4096 --frames 1024 --iters 2 > gpurun_out/r03an_$arm$r.json 2>/dev/null || exit 1
  else timeout -k 10 300 python3 tools/ab_run.py --lib-dir ab_$arm tools/lg_bench.py --pairs 4096 --frames 1024 --iters 2 > gpurun_out/r03an_$arm$r.json 2>/dev/null || exit 1; fi
  echo $arm $(tail -1 gpurun_out/r03an_$arm$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_call'], d['ffn_fused'], d['matches_mean'])")
done
done
