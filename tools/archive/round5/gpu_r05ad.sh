#!/bin/bash
# Round-5 GPU batch ad (the PMC half of batch ac, whose determinism probe call lacked its library argument): attention staging writes by the calibrated write rule (tree, MLG_ATT_STAGE_W)
# vs the round-4 staging (ab_att/w0): attention / LightGlue / ViT GPU tests, LightGlue stage bench
# (digest, attention ms) and ViT bench (descriptor hash) ABAB, attention determinism probe, then
# one PMC pass per arm for the attention's LDS conflict share.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u tools/attn_det_probe.py multi-level-indoor-slam_amd/mlgate > "$O/r05ad_det.log" 2>&1 || { tail -5 "$O/r05ad_det.log"; exit 1; }
echo "det $(tail -1 "$O/r05ad_det.log" | cut -c1-400)"
cd /tmp && export TMPDIR=/tmp
for arm in tree w0; do
  pre=""; [ $arm != tree ] && pre="$R/tools/ab_run.py --lib-dir $R/ab_att/w0"
  timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
      --output-format csv -d /tmp/pmc_ad_$arm/pass1 -o run -- python3 $pre "$R/tools/lg_bench.py" --pairs 512 --iters 1 > "$O/r05ad_pmc_$arm.log" 2>&1 \
      || { echo "pmc $arm failed"; tail -3 "$O/r05ad_pmc_$arm.log"; exit 1; }
  python3 "$R/tools/pmc_summary.py" /tmp/pmc_ad_$arm k_attention > "$O/r05ad_pmc_$arm.txt" 2>&1
  echo "== $arm"; cut -c1-330 "$O/r05ad_pmc_$arm.txt"
done
