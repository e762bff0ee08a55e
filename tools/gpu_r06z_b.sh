#!/bin/bash
# Round-6 final evidence, part B: the bench-scale fp32 chain fixture regenerated on the final
# RANSAC (explicit-fma Aberth iteration in both twins), with GPU RANSAC vs C twin on every
# ordered pair of the step (product lists and fp32-chain lists).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 1000 python -u tools/bench_parity.py chain --out "$O/r06z_bench_chain_fp32.npz" --workers 15 > "$O/r06z_chain.log" 2>&1
rc=$?; grep -v amdgpu.ids "$O/r06z_chain.log" | tail -c 2500; exit $rc
