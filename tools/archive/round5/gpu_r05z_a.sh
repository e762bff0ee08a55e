#!/bin/bash
# Round-5 final evidence, part A: the whole GPU suite, smoke, the default bench line.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 120 tools/bin/occupancy_probe > "$O/r05z_occupancy.txt" 2>&1 || { cat "$O/r05z_occupancy.txt"; exit 1; }
cat "$O/r05z_occupancy.txt"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$O/r05z_pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/r05z_pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/r05z_smoke.log" 2>&1
rc=$?; tail -2 "$O/r05z_smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > "$O/r05z_bench.json" 2> "$O/r05z_bench.err"
rc=$?; tail -c 400 "$O/r05z_bench.json"; exit $rc
