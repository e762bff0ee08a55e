#!/bin/bash
# r03o: HEAD evidence after the session restart -- new SALAD tests (non-blocking), full GPU suite, smoke,
# default bench (LoFTR + cpu baseline), rocprof stats
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_salad_gpu.py tests/test_orb_gpu.py -v --timeout 200 --timeout-method thread > gpurun_out/r03o_salad.log 2>&1; rc=$?; tail -3 gpurun_out/r03o_salad.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --deselect tests/test_salad_gpu.py --deselect tests/test_orb_gpu.py --timeout 250 --timeout-method thread > gpurun_out/r03o_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03o_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03o_smoke.log 2>&1 || { tail -5 gpurun_out/r03o_smoke.log; exit 1; }
tail -2 gpurun_out/r03o_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r03o_bench.json 2> gpurun_out/r03o_bench.err || { tail -5 gpurun_out/r03o_bench.err; exit 1; }
tail -c 400 gpurun_out/r03o_bench.json
timeout -k 10 700 bash tools/gpu_profile.sh r03o
