#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters in this pass).
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r1}"
OUT="$REPO/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$REPO/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_stdout.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 "$OUT/bench_stdout.log"
find "$OUT" -name "*stats*" | head
exit $rc
