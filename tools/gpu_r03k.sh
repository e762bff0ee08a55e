#!/bin/bash
# r03k: LoFTR single-pass statistics / batched KV loads / vector FPN merge; decision-sample GPU test
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_loftr_gpu.py tests/test_decisions_gpu.py -x -v --timeout 250 --timeout-method thread > gpurun_out/r03k_tests.log 2>&1; rc=$?; tail -4 gpurun_out/r03k_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_loftr_k -o loftr -- python3 tools/loftr_bench.py --frames 32 --pairs 32 > gpurun_out/r03k_prof.log 2>&1 || { tail -5 gpurun_out/r03k_prof.log; exit 1; }
grep '^{' gpurun_out/r03k_prof.log | tail -1
