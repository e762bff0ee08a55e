#!/bin/bash
# r04t: LightGlue projections in 4-wave half-part workgroups, two per CU (MLG_PROJ_RES=2):
# LightGlue kernel tests with that build, then the stage bench ABAB against the tree
set -u
mkdir -p gpurun_out
PT=/usr/local/lib/python3.10/dist-packages/pytest/__main__.py
timeout -k 10 400 python -u tools/ab_run.py --lib-dir ab_proj2 $PT -x -v --timeout 300 --timeout-method thread -m gpu tests/test_lightglue_gpu.py tests/test_kernels_gpu.py tests/test_pipeline_gpu.py > gpurun_out/r04t_pytest_proj2.log 2>&1
rc=$?; echo "pytest(proj2) rc=$rc"; tail -2 gpurun_out/r04t_pytest_proj2.log
[ $rc = 0 ] || exit $rc
for arm in tree proj2 tree proj2; do
  if [ $arm = tree ]; then timeout -k 10 240 python -u tools/lg_bench.py --pairs 2048 --iters 2 >> gpurun_out/r04t_lg_$arm.log 2>&1 || exit 1
  else timeout -k 10 240 python -u tools/ab_run.py --lib-dir ab_proj2 tools/lg_bench.py --pairs 2048 --iters 2 >> gpurun_out/r04t_lg_$arm.log 2>&1 || exit 1; fi
  echo "lg $arm $(grep '^{' gpurun_out/r04t_lg_$arm.log | tail -1 | cut -c1-330)"
done
