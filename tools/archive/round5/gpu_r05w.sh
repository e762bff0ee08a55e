#!/bin/bash
# Round-5 GPU batch w: where the projection's LDS "bank conflict" cycles come from.  PMC of the
# resident (non-pipelined) form with one stream removed at a time (MLG_PROJ_PROBE builds,
# results wrong by design): res = all streams, nodma = no LDS-DMA of the next tile (4),
# noepi = no epilogue / staging / copy-out (2), nogemm = no GEMM x-fragment reads (1); tree = product.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for arm in tree res nodma noepi nogemm; do
  pre=""; [ $arm != tree ] && pre="$R/tools/ab_run.py --lib-dir $R/ab_pp/$arm"
  timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
      --output-format csv -d /tmp/pmc_w_$arm/pass1 -o run -- python3 $pre "$R/tools/proj_pipe_check.py" --iters 2 > "$O/r05w_pmc_$arm.log" 2>&1 \
      || { echo "pmc $arm failed"; tail -3 "$O/r05w_pmc_$arm.log"; exit 1; }
  python3 "$R/tools/pmc_summary.py" /tmp/pmc_w_$arm k_lg_proj > "$O/r05w_pmc_$arm.txt" 2>&1
  echo "== $arm"; cut -c1-330 "$O/r05w_pmc_$arm.txt"
done
