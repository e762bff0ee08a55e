#!/bin/bash
# r04a: bench-scale retrieval parity vs fp32 descriptors + oracle timing probe
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/bench_parity.py retrieval --out gpurun_out/r04a_retrieval.npz > gpurun_out/r04a_retrieval.log 2>&1 || { tail -20 gpurun_out/r04a_retrieval.log; exit 1; }
tail -1 gpurun_out/r04a_retrieval.log
timeout -k 10 300 python -u tools/bench_parity.py probe > gpurun_out/r04a_probe.log 2>&1 || { tail -20 gpurun_out/r04a_probe.log; exit 1; }
tail -1 gpurun_out/r04a_probe.log
