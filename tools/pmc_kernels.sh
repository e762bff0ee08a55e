#!/bin/bash
# Attributed PMC passes (one rocprofv3 --pmc run per pass, never combined with tracing) over
# the LightGlue stage (tools/lg_bench.py) and the ViT forward (tools/vit_bench.py);
# summarised per kernel by tools/pmc_summary.py.   bash tools/pmc_kernels.sh <tag>
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-x}"
cd /tmp && export TMPDIR=/tmp
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"
for wl in lg vit; do
  OUT="$REPO/gpurun_out/pmc_${TAG}_${wl}"
  mkdir -p "$OUT"
  if [ $wl = lg ]; then CMD="$REPO/tools/lg_bench.py --pairs 1024 --iters 1"; else CMD="$REPO/tools/vit_bench.py --iters 1"; fi
  i=0
  for pass in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 180 rocprofv3 --pmc $pass --output-format csv -d "$OUT/pass$i" -o run -- python3 $CMD > "$OUT/pass$i.log" 2>&1
    rc=$?; echo "$wl pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/pass$i.log"; exit $rc; fi
  done
  python3 "$REPO/tools/pmc_summary.py" "$OUT" > "$REPO/gpurun_out/pmc_${TAG}_${wl}.txt"
  head -40 "$REPO/gpurun_out/pmc_${TAG}_${wl}.txt"
done
