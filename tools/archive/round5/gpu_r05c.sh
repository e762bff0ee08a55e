#!/bin/bash
# Round-5 GPU batch c: LDS conflict calibration (PMC), FFN zero-C A/B, per-rank projection.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE \
    --output-format csv -d "$O/r05c_lds" -o lds -- "$R/tools/bin/lds_probe" > "$O/r05c_lds.log" 2>&1 || exit 1
echo "lds probe ok"
cd "$R"
tools/gpu_ab.sh ab_ffn_base r05c_ffn 2 -- tools/lg_bench.py --pairs 2048 --iters 2 > "$O/r05c_ffn_ab.txt" 2>&1 || { cat "$O/r05c_ffn_ab.txt"; exit 1; }
cat "$O/r05c_ffn_ab.txt"
timeout -k 10 600 python -u tools/rank_projection.py > "$O/r05c_rank.log" 2>&1 || { tail -5 "$O/r05c_rank.log"; exit 1; }
tail -3 "$O/r05c_rank.log"
