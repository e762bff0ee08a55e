#!/bin/bash
# Round 6: the whole GPU suite, smoke and the default bench line after the RANSAC twin change.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"; P="${1:-r06b}"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$O/${P}_pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/${P}_pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/${P}_smoke.log" 2>&1
rc=$?; tail -2 "$O/${P}_smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > "$O/${P}_bench.json" 2> "$O/${P}_bench.err"
rc=$?; tail -c 600 "$O/${P}_bench.json"; exit $rc
