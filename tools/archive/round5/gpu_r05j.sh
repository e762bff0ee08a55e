#!/bin/bash
# Round-5 GPU batch j: FFN phase timeline (MLG_FFN_TRACE build) at 2 M and 21 M tokens.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
for m in 2097152 20971520; do
  timeout -k 10 300 python -u tools/ab_run.py --lib-dir ab_ffnt tools/ffn_trace.py --tokens $m > "$O/r05j_trace_$m.log" 2>&1 || { tail -5 "$O/r05j_trace_$m.log"; exit 1; }
  grep '^{' "$O/r05j_trace_$m.log"
done
