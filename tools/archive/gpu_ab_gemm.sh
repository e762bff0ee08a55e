#!/bin/bash
# HISTORICAL (kept as the recipe of the profiles it produced): it switches arms through
# runtime knobs (MLG_FFN_* / MLG_PROJ_* / MLG_GEMM_VARIANT env vars, MLGATE_LIB_DIR) that the
# library no longer reads, so both arms would now run the same build.  Build each arm
# with -D flags instead and load it through tools/ab_run.py --lib-dir (tools/gpu_r03ag.sh).
echo "$0: historical recipe; its runtime A/B knobs are gone (see header)" >&2; exit 2
# GEMM variant 5 (4-deep BK=32 ring) vs 4 (2-deep BK=64): kernel tests, the GEMM
# microbench, and the bench with MLG_GEMM_VARIANT=5 / 4 on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/gemm_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/gemm_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python3 tools/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1
rc=$?; echo "gemm_bench rc=$rc"; head -3 gpurun_out/gemm_bench.log | grep -v amdgpu.ids | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
for v in 5 4; do
  MLG_GEMM_VARIANT=$v timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/gemm_benchpy_$v.log 2>&1
  rc=$?; echo "bench variant=$v rc=$rc"; tail -1 gpurun_out/gemm_benchpy_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']['stage_ms_per_step']; print(d['value'], d['ms_per_step'], {k: r[k] for k in r if k.startswith('vit')}, d['config']['false_loop_closure_rejections']['total'])"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
