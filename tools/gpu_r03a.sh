#!/bin/bash
# r03a: LightGlue co-scheduling determinism, pre-fix build (ab_prefix/) vs the in-tree build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_run.py --lib-dir ab_prefix tools/lg_determinism.py > gpurun_out/r03a_prefix.log 2>&1 || { echo "prefix arm failed: $?"; tail -20 gpurun_out/r03a_prefix.log; exit 1; }
timeout -k 10 300 python -u tools/lg_determinism.py > gpurun_out/r03a_fixed.log 2>&1 || { echo "fixed arm failed: $?"; tail -20 gpurun_out/r03a_fixed.log; exit 1; }
grep summary gpurun_out/r03a_prefix.log gpurun_out/r03a_fixed.log
