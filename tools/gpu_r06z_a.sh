#!/bin/bash
# Round-6 final evidence, part A: every GPU test, smoke(), and the default bench line.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"; T="${1:-r06z}"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/${T}_gpu_tests.log" 2>&1
rc=$?; tail -3 "$O/${T}_gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/${T}_smoke.log" 2>&1
rc=$?; tail -2 "$O/${T}_smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > "$O/${T}_bench.json" 2> "$O/${T}_bench.err"
rc=$?; tail -c 400 "$O/${T}_bench.json"; exit $rc
