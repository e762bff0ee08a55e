#!/bin/bash
set -u
REPO="${GRAFT_REPO_ROOT}"
OUT="$REPO/gpurun_out/prof_ransac"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$REPO/tools/ransac_bench.py" "$@" > "$OUT/stdout.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 "$OUT/stdout.log"
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(f'{float(r["AverageNs"])/1e3:10.1f} us x {r["Calls"]:>5}  {r["Name"][:80]}')
PY
exit $rc
