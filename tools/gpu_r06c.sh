#!/bin/bash
# Round 6: regenerate the bench-scale fp32 chain fixture with the bit-exact RANSAC twin, and
# report GPU RANSAC vs C twin on every ordered pair of a bench step (product lists and the
# fp32 chain's lists).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 1100 python -u tools/bench_parity.py chain --out "$O/r06c_bench_chain_fp32.npz" --workers 15 > "$O/r06c_chain.log" 2>&1
rc=$?; grep -v amdgpu.ids "$O/r06c_chain.log" | tail -c 3000; exit $rc
