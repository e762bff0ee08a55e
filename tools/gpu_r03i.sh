#!/bin/bash
# r03i: LoFTR per-kernel profile (backbone + matching) for configs[4]
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_loftr -o loftr -- python3 tools/loftr_bench.py --frames 32 --pairs 32 > gpurun_out/r03i_loftr.log 2>&1 || { tail -5 gpurun_out/r03i_loftr.log; exit 1; }
tail -1 gpurun_out/r03i_loftr.log
f=$(find gpurun_out/prof_loftr -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r03i_loftr_kernel_stats.csv
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open("gpurun_out/r03i_loftr_kernel_stats.csv")))
for r in rows[:25]:
    print(r["Name"][:90], r["Calls"], r["TotalDurationNs"], r["AverageNs"], r["Percentage"])
PY
