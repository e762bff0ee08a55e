#!/bin/bash
# r03h: new GPU tests (batched rerank, k > 4096, float labels), full GPU suite, smoke, LoFTR timing
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_retrieval_gpu.py tests/test_pipeline_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r03h_new.log 2>&1; rc=$?; tail -3 gpurun_out/r03h_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03h_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03h_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03h_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r03h_smoke.log
timeout -k 10 300 python -u tools/loftr_bench.py --frames 32 --pairs 32 > gpurun_out/r03h_loftr.json 2>&1 || exit 1
tail -1 gpurun_out/r03h_loftr.json
