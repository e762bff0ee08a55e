#!/bin/bash
# HBM traffic per launch of the LightGlue kernels: two PMC passes (FETCH_SIZE, WRITE_SIZE;
# never combined with tracing), each its own rocprofv3 run of tools/lg_bench.py (one
# $PAIRS-pair LightGlue call = bench.py's lg_chunk; a --pmc pass over the whole bench
# segfaulted inside the profiler), then tools/pmc_traffic.py writes
# profiles/pmc_traffic.json (bench.py's roofline.traffic).
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc_traffic"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for pass in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $pass --output-format csv -d "$OUT/pass$i" -o run -- \
      python3 "$REPO/tools/lg_bench.py" --iters 1 --pairs ${PAIRS:-4096} --frames ${FRAMES:-1024} > "$OUT/pass$i.log" 2>&1
  rc=$?; echo "pass $i ($pass) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 "$REPO/tools/pmc_traffic.py" "$OUT" "$OUT/pmc_traffic.json"  # copy to profiles/ after the merge
