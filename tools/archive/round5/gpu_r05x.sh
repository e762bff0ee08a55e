#!/bin/bash
# Round-5 GPU batch x: LDS calibration of the paired projection staging streams (tools/lds_probe.hip
# patterns 29-35) beside the round-5 calibration set; summaries only.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE \
    --output-format csv -d /tmp/r05x_lds -o lds -- "$R/tools/bin/lds_probe" > "$O/r05x_lds.log" 2>&1 || { tail -5 "$O/r05x_lds.log"; exit 1; }
f=$(find /tmp/r05x_lds -name '*counter_collection.csv' | head -1); cp "$f" "$O/r05x_lds_counters.csv"; echo "lds probe ok"
