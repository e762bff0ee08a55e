#!/bin/bash
# r03g: no-SLP build -- GPU tests, LightGlue co-scheduling determinism, bench, decision sample
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03g_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03g_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lg_determinism.py --modes single,threads2,noise > gpurun_out/r03g_determinism.log 2>&1 || exit 1
grep summary gpurun_out/r03g_determinism.log
timeout -k 10 400 python -u bench.py > gpurun_out/r03g_bench.json 2> gpurun_out/r03g_bench.err || exit 1
tail -c 600 gpurun_out/r03g_bench.json
timeout -k 10 300 python -u tools/decision_sample.py --out gpurun_out/decision_sample.npz > gpurun_out/r03g_decision.log 2>&1 || exit 1
tail -1 gpurun_out/r03g_decision.log
timeout -k 10 600 bash tools/pmc_kernels.sh r03g > gpurun_out/r03g_pmc.log 2>&1 || { tail -5 gpurun_out/r03g_pmc.log; exit 1; }
grep -E "k_attention_varlen|k_lg_ffn|k_lg_proj|k_gemm256|k_attention " gpurun_out/pmc_r03g_*.txt | grep mfma_util | head -20
