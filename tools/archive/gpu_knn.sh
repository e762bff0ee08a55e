#!/bin/bash
# kNN: parity tests, timing, rocprof kernel stats and one FETCH_SIZE / WRITE_SIZE pass each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/knn
timeout -k 10 300 python -u -m pytest tests/test_retrieval_gpu.py tests/test_api_gpu.py tests/test_pipeline_gpu.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/knn/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/knn/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python tools/knn_bench.py || exit $?
timeout -k 10 120 python tools/knn_bench.py --n 19163 --k 10 --iters 5 || exit $?
REPO=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/knn/trace -o run -- python3 $REPO/tools/knn_bench.py > /dev/null 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $REPO/gpurun_out/knn/fetch -o run -- python3 $REPO/tools/knn_bench.py --iters 2 > /dev/null 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $REPO/gpurun_out/knn/write -o run -- python3 $REPO/tools/knn_bench.py --iters 2 > /dev/null 2>&1 || exit $?
echo pmc done
