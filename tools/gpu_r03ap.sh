#!/bin/bash
# r03ap(b): k_asg_arg reading S straight from global / L2 (MLG_ASG_DIRECT=1, +unroll 4) vs the LDS-staged tile (tree): rocprof kernel stats of
# tools/lg_bench.py (4096 pairs) per arm; matches must be identical
set -u
REPO="$(pwd)"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for arm in tree dir diru; do
  OUT="$REPO/gpurun_out/r03ap_$arm"; mkdir -p "$OUT"
  if [ $arm = tree ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 "$REPO/tools/lg_bench.py" --pairs 4096 --frames 1024 --iters 2 > "$OUT/out.json" 2> "$OUT/err.log" || { tail -3 "$OUT/err.log"; exit 1; }
  else
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 "$REPO/tools/ab_run.py" --lib-dir "$REPO/ab_$arm" "$REPO/tools/lg_bench.py" --pairs 4096 --frames 1024 --iters 2 > "$OUT/out.json" 2> "$OUT/err.log" || { tail -3 "$OUT/err.log"; exit 1; }
  fi
  S=$(find "$OUT" -name "*kernel_stats.csv" | head -1)
  echo "$arm $(grep -h '{' "$OUT/out.json" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_call'], d['matches_mean'])") $(grep -E 'k_asg_arg\(|k_asg_sim' "$S" | awk -F'","' '{print $0}' | python3 -c "
import sys,csv
for row in csv.reader(sys.stdin): print(row[0][24:36], row[1], round(float(row[3])/1000,1), end='; ')")"
done
