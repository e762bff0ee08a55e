#!/bin/bash
# Round 6, first GPU call: RANSAC bit-exactness against the C twin (tests) and the cost of
# building ransac.hip without FP contraction (same-box A/B of tools/ransac_bench.py):
#   rs_old     the round-5 source, contraction on
#   rs_newfast this round's source (shared rs_math.h) with contraction forced on
#   product    this round's build (-ffp-contract=off)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_ransac_gpu.py tests/test_oracle_geometry.py -x -v \
    --timeout 300 --timeout-method thread > gpurun_out/r06a_pytest.log 2>&1
echo "pytest exit $?"
tail -3 gpurun_out/r06a_pytest.log
for rep in 0 1; do
  for arm in rs_old rs_newfast product; do
    for cfg in "--pairs 5000 --matches 600 --inliers 0.2" "--pairs 2000 --matches 1200 --inliers 0.5"; do
      if [ "$arm" = product ]; then
        out=$(timeout -k 10 120 python tools/ransac_bench.py $cfg) || { echo "bench failed $arm"; exit 1; }
      else
        out=$(timeout -k 10 120 python tools/ab_run.py --lib-dir ab/$arm tools/ransac_bench.py $cfg) || { echo "bench failed $arm"; exit 1; }
      fi
      echo "$arm $rep $out" | tee -a gpurun_out/r06a_ransac_ab.txt
    done
  done
done
