#!/bin/bash
# r04v: split ViT attention -- waves with no live query skip their compute (tree / ab_idle)
# vs not (ab_base): ViT tests on the tree, then vit_bench ABAB
set -u
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_vit_gpu.py tests/test_kernels_gpu.py > gpurun_out/r04v_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r04v_pytest.log
[ $rc = 0 ] || exit $rc
for arm in base idle base idle; do
  timeout -k 10 200 python -u tools/ab_run.py --lib-dir ab_$arm tools/vit_bench.py --vit split >> gpurun_out/r04v_vit_$arm.log 2>&1 || exit 1
  echo "vit $arm $(grep '^{' gpurun_out/r04v_vit_$arm.log | tail -1 | cut -c1-120) $(grep -o '"attention": {[^}]*}' gpurun_out/r04v_vit_$arm.log | tail -1)"
done
