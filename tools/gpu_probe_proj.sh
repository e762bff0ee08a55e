#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for p in ${PROBES:-0 1 2 3 4 5 6 8 0}; do
  MLG_PROJ_PROBE=$p timeout -k 10 120 python3 tools/proj_ab.py --iters 10 > gpurun_out/probe_$p.log 2>&1
  rc=$?; echo "probe=$p rc=$rc $(tail -1 gpurun_out/probe_$p.log | cut -c1-90)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
