#!/bin/bash
# HISTORICAL (kept as the recipe of the profiles it produced): it switches arms through
# runtime knobs (MLG_FFN_* / MLG_PROJ_* / MLG_GEMM_VARIANT env vars, MLGATE_LIB_DIR) that the
# library no longer reads, so both arms would now run the same build.  Build each arm
# with -D flags instead and load it through tools/ab_run.py --lib-dir (tools/gpu_r03ag.sh).
echo "$0: historical recipe; its runtime A/B knobs are gone (see header)" >&2; exit 2
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for p in ${PROBES:-0 1 2 3 4 5 6 8 0}; do
  MLG_PROJ_PROBE=$p timeout -k 10 120 python3 tools/proj_ab.py --iters 10 > gpurun_out/probe_$p.log 2>&1
  rc=$?; echo "probe=$p rc=$rc $(tail -1 gpurun_out/probe_$p.log | cut -c1-90)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
