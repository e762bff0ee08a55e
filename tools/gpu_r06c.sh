#!/bin/bash
# Round 6: the GPU suite on the ABI-3 build, then the bench-scale fp32 chain fixture
# regenerated with the bit-exact RANSAC twin, reporting GPU RANSAC vs C twin on every
# ordered pair of a bench step (product lists and the fp32 chain's lists).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$O/r06c_pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/r06c_pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/bench_parity.py chain --out "$O/r06c_bench_chain_fp32.npz" --workers 15 > "$O/r06c_chain.log" 2>&1
rc=$?; grep -v amdgpu.ids "$O/r06c_chain.log" | tail -c 3000; exit $rc
