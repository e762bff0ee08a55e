#!/bin/bash
# Round-5 GPU batch d: LDS write-rule calibration; the new GPU tests of this round.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE \
    --output-format csv -d "$O/r05d_lds" -o lds -- "$R/tools/bin/lds_probe" > "$O/r05d_lds.log" 2>&1 || exit 1
echo "lds probe ok"
cd "$R"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ransac_gpu.py \
    tests/test_loftr_gpu.py tests/test_vit_gpu.py tests/test_api_gpu.py tests/test_pipeline_gpu.py \
    > "$O/r05d_pytest.log" 2>&1
rc=$?; tail -15 "$O/r05d_pytest.log"; exit $rc
