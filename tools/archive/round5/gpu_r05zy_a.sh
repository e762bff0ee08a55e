#!/bin/bash
# Round-5 final evidence, final (after the assignment full-tile scans), part A: the whole GPU suite, smoke, the default bench line.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$O/r05zy_pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/r05zy_pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/r05zy_smoke.log" 2>&1
rc=$?; tail -2 "$O/r05zy_smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > "$O/r05zy_bench.json" 2> "$O/r05zy_bench.err"
rc=$?; tail -c 400 "$O/r05zy_bench.json"; exit $rc
