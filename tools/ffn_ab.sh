#!/bin/bash
# FFN launch-form A/B on one box (tools/proj_ab.py; MLG_FFN_GRID = workgroups per CU of
# the persistent grid, 0 = one workgroup per tile).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for g in 0 2 0 2; do
  MLG_FFN_GRID=$g timeout -k 10 120 python3 tools/proj_ab.py --iters 10 > gpurun_out/ffn_ab_$g.log 2>&1
  rc=$?; echo "grid=$g rc=$rc $(grep -o '"lg_ffn_ms": [0-9.]*' gpurun_out/ffn_ab_$g.log) $(grep -o '"gemm_512x512_gelu_ms": [0-9.]*' gpurun_out/ffn_ab_$g.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
