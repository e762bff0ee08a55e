#!/bin/bash
# Round 6: the bench-scale chain re-run with the model-bit check (GPU RANSAC vs the C twin:
# counts, masks and model bits on every ordered pair of a bench step, product and fp32 lists).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 1000 python -u tools/bench_parity.py chain --out "$O/r06v_bench_chain_fp32.npz" --workers 15 > "$O/r06v_chain.log" 2>&1
rc=$?; grep -v amdgpu.ids "$O/r06v_chain.log" | tail -c 2500; exit $rc
