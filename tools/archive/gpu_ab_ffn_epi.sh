#!/bin/bash
# HISTORICAL (kept as the recipe of the profiles it produced): it switches arms through
# runtime knobs (MLG_FFN_* / MLG_PROJ_* / MLG_GEMM_VARIANT env vars, MLGATE_LIB_DIR) that the
# library no longer reads, so both arms would now run the same build.  Build each arm
# with -D flags instead and load it through tools/ab_run.py --lib-dir (tools/gpu_r03ag.sh).
echo "$0: historical recipe; its runtime A/B knobs are gone (see header)" >&2; exit 2
# Prices the fused FFN's LayerNorm + GELU epilogue: the same launch with ReLU instead
# (MLG_FFN_PROBE_RELU=1; wrong results, timing only) vs LightGlue's epilogue.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 0 1 0; do
  MLG_FFN_PROBE_RELU=$r timeout -k 10 120 python3 tools/proj_ab.py --iters 10 > gpurun_out/ffnepi_$r.log 2>&1
  rc=$?; echo "probe_relu=$r rc=$rc $(grep -o '"lg_ffn_ms": [0-9.]*' gpurun_out/ffnepi_$r.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
