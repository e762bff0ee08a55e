#!/bin/bash
# Round 6: same-box ABAB of the ViT forward, round-5 attention.hip + gemm_bf16.hip (ab/vit_r05)
# against the tree (split attention O epilogue b128 pairs, lo V^T tile 8 B off so no
# ds_read2st64 fusion, split-GEMM staged-epilogue half flip), digests compared; then the
# tree's ViT PMC passes (LDS conflict shares).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
bash tools/gpu_ab.sh ab/vit_r05 r06e 3 -- tools/vit_bench.py --frames 492 --batch 246 --iters 2 | tee gpurun_out/r06e_ab_vit.txt
[ ${PIPESTATUS[0]} -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
OUT="$R/gpurun_out/pmc_r06e_vit"; mkdir -p "$OUT"
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"
i=0
for pass in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $pass --output-format csv -d "$OUT/pass$i" -o run -- python3 "$R/tools/vit_bench.py" --iters 1 > "$OUT/pass$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/pass$i.log"; exit $rc; }
done
python3 "$R/tools/pmc_summary.py" "$OUT" > "$R/gpurun_out/pmc_r06e_vit.txt"
rm -rf "$OUT"
grep -v "^    {" "$R/gpurun_out/pmc_r06e_vit.txt" | grep "k_gemm256s\|k_attention\|preprocess"
