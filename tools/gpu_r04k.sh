#!/bin/bash
# r04k: RANSAC unused-slot fix (mixed small pairs, LoFTR sharded gate), split-GELU poly,
# then the whole GPU suite and the default bench
set -u
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 200 $T tests/test_ransac_gpu.py > gpurun_out/r04k_ransac.log 2>&1 && echo "ransac ok" &&
timeout -k 10 300 $T "tests/test_distributed_gpu.py::test_sharded_gate_equals_single_rank[loftr]" > gpurun_out/r04k_loftr.log 2>&1 && echo "loftr ok" &&
timeout -k 10 600 $T -m gpu tests > gpurun_out/r04k_pytest_gpu.log 2>&1 && echo "suite ok" &&
timeout -k 10 400 python -u bench.py > gpurun_out/r04k_bench.json 2> gpurun_out/r04k_bench.err && echo "bench ok"
rc=$?
echo "rc=$rc"
if [ $rc = 0 ]; then
  # FFN SLP probe: does the drift follow the rsqrt fix-up packed into v_pk_mul_f32?
  for arm in ctl slp slprsq1 slprsq2; do
    timeout -k 10 240 python -u tools/ab_run.py --lib-dir ab_ffn_$arm tools/ffn_interference.py --victims ffn --partners attn,proj --repeats 12 > gpurun_out/r04k_ffn_$arm.log 2>&1 || { rc=$?; echo "ffn $arm rc=$rc"; break; }
    echo "$arm $(tail -1 gpurun_out/r04k_ffn_$arm.log)"
  done
fi
if [ $rc = 0 ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04k_lfprof -o lf -- python3 tools/loftr_bench.py --pairs 64 > gpurun_out/r04k_loftr_bench.log 2>&1; echo "loftr prof rc=$?"
fi
exit $rc
for f in gpurun_out/r04k_ransac.log gpurun_out/r04k_loftr.log gpurun_out/r04k_pytest_gpu.log; do tail -4 $f 2>/dev/null; done
cat gpurun_out/r04k_bench.json 2>/dev/null | head -c 600
