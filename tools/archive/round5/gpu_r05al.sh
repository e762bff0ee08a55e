#!/bin/bash
# Round-5 GPU batch al: the bench with SuperPoint batches of 256 keyframes vs the default 64 (ABAB, 2 timed
# steps each; rejections must be identical: per-frame SuperPoint results do not depend on the batch).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
for rep in 0 1; do
  for b in 64 256; do
    timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --sp-batch $b > "$O/r05al_b${b}_$rep.json" 2> "$O/r05al_b${b}_$rep.err" \
      || { echo "bench sp_batch $b failed"; tail -5 "$O/r05al_b${b}_$rep.err"; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['false_loop_closure_rejections']['total'], d['roofline']['frac'])" "$O/r05al_b${b}_$rep.json" "sp_batch=$b rep $rep"
  done
done
