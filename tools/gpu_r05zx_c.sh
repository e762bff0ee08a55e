#!/bin/bash
# Round-5 final evidence, part C: the default bench line once more on another box (box-to-box spread).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u bench.py > "$O/r05zx_bench2.json" 2> "$O/r05zx_bench2.err"
rc=$?; tail -c 300 "$O/r05zx_bench2.json"; exit $rc
