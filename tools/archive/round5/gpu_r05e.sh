#!/bin/bash
# Round-5 GPU batch e: LDS write-rule calibration; the whole GPU suite; A/B of the rotary
# factor layout (LightGlue stage bench) and the split-bf16 LoFTR similarity vs ab_base_r05.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE \
    --output-format csv -d "$O/r05e_lds" -o lds -- "$R/tools/bin/lds_probe" > "$O/r05e_lds.log" 2>&1 || exit 1
echo "lds probe ok"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$O/r05e_pytest.log" 2>&1
rc=$?; tail -5 "$O/r05e_pytest.log"; [ $rc -eq 0 ] || exit $rc
tools/gpu_ab.sh ab_base_r05 r05e_lg 2 -- tools/lg_bench.py --pairs 2048 --iters 2 > "$O/r05e_lg_ab.txt" 2>&1 || { cat "$O/r05e_lg_ab.txt"; exit 1; }
cat "$O/r05e_lg_ab.txt"
tools/gpu_ab.sh ab_base_r05 r05e_lf 2 -- tools/loftr_bench.py --frames 64 --pairs 64 > "$O/r05e_lf_ab.txt" 2>&1 || { cat "$O/r05e_lf_ab.txt"; exit 1; }
cat "$O/r05e_lf_ab.txt"
