#!/bin/bash
# HISTORICAL (kept as the recipe of the profiles it produced): it switches arms through
# runtime knobs (MLG_FFN_* / MLG_PROJ_* / MLG_GEMM_VARIANT env vars, MLGATE_LIB_DIR) that the
# library no longer reads, so both arms would now run the same build.  Build each arm
# with -D flags instead and load it through tools/ab_run.py --lib-dir (tools/gpu_r03ag.sh).
echo "$0: historical recipe; its runtime A/B knobs are gone (see header)" >&2; exit 2
# FFN launch-form A/B on one box (tools/proj_ab.py; MLG_FFN_GRID = workgroups per CU of
# the persistent grid, 0 = one workgroup per tile).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for g in 0 2 0 2; do
  MLG_FFN_GRID=$g timeout -k 10 120 python3 tools/proj_ab.py --iters 10 > gpurun_out/ffn_ab_$g.log 2>&1
  rc=$?; echo "grid=$g rc=$rc $(grep -o '"lg_ffn_ms": [0-9.]*' gpurun_out/ffn_ab_$g.log) $(grep -o '"gemm_512x512_gelu_ms": [0-9.]*' gpurun_out/ffn_ab_$g.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
