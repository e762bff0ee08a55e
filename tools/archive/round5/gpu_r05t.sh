#!/bin/bash
# Round-5 GPU batch t: the projection LDS conflict share, tree (MLG_PROJ_STAGE2) vs ab_proj/s0
# (batch s's PMC pass wrote no pass*/ directory, so its summaries were empty).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for arm in tree s0; do
  pre=""; [ $arm != tree ] && pre="$R/tools/ab_run.py --lib-dir $R/ab_proj/$arm"
  timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
      --output-format csv -d /tmp/pmc_t_$arm/pass1 -o run -- python3 $pre "$R/tools/proj_pipe_check.py" --iters 2 > "$O/r05t_pmc_$arm.log" 2>&1 \
      || { echo "pmc $arm failed"; tail -3 "$O/r05t_pmc_$arm.log"; exit 1; }
  python3 "$R/tools/pmc_summary.py" /tmp/pmc_t_$arm k_lg_proj > "$O/r05t_pmc_$arm.txt" 2>&1
  echo "== $arm"; cut -c1-300 "$O/r05t_pmc_$arm.txt"
done
