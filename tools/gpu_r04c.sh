#!/bin/bash
# r04c: whole bench step vs the fp32 chain (retrieval + every verified pair)
set -u
mkdir -p gpurun_out
timeout -k 10 1130 python -u tools/bench_parity.py chain --workers 15 --out gpurun_out/r04c_chain.npz > gpurun_out/r04c_chain.log 2>&1 || { tail -20 gpurun_out/r04c_chain.log; exit 1; }
tail -2 gpurun_out/r04c_chain.log
