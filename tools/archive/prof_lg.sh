#!/bin/bash
# rocprofv3 kernel stats of the LightGlue stage microbenchmark (tools/lg_bench.py).
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/prof_lg_${1:-x}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$REPO/tools/lg_bench.py" ${LG_ARGS:-} > "$OUT/stdout.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; grep pairs "$OUT/stdout.log"
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:24]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['Percentage']):5.1f}% n={r['Calls']:>5} avg={float(r['AverageNs'])/1e3:8.1f}us {r['Name'][:90]}")
PY
exit $rc
