#!/bin/bash
# r03ag: attention tile A/B through tools/ab_run.py --lib-dir (tree = HEAD):
#   ab_dot2: row sums as v_dot2c_f32_bf16 over the packed P pair
#   ab_p1 / ab_p2: timing-only probes (row-sum adds removed / v_exp removed; wrong results)
set -u
mkdir -p gpurun_out
for r in 1 2; do
for arm in tree dot2 p1 p2; do
  if [ $arm = tree ]; then timeout -k 10 120 python3 tools/attn_bench.py --pairs 1024 --iters 5 > gpurun_out/r03ag_attn_$arm$r.log 2>&1 || exit 1
  else timeout -k 10 120 python3 tools/ab_run.py --lib-dir ab_$arm tools/attn_bench.py --pairs 1024 --iters 5 > gpurun_out/r03ag_attn_$arm$r.log 2>&1 || exit 1; fi
  echo "attn $arm $(tail -1 gpurun_out/r03ag_attn_$arm$r.log)"
done
done
for arm in tree dot2; do
  if [ $arm = tree ]; then timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03ag_bench_$arm.log 2>&1 || exit 1
  else timeout -k 10 400 python3 tools/ab_run.py --lib-dir ab_$arm bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03ag_bench_$arm.log 2>&1 || exit 1; fi
  echo "bench $arm"; tail -1 gpurun_out/r03ag_bench_$arm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['stage_ms_per_step']['lightglue_attention'], d['config']['false_loop_closure_rejections']['total'])"
done
