#!/bin/bash
# Round-5 GPU batch af: the split GEMM's staged bf16-pair epilogue as paired b128 writes (tree,
# MLG_GEMM_STAGE_W, v_permlane16_swap) vs per-half b64 (ab_gemm/w0): ViT / kernel GPU tests,
# ViT bench (descriptor hash, fc1 / qkv ms) ABAB, then a PMC pass per arm over the ViT forward.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_vit_gpu.py tests/test_retrieval_gpu.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > "$O/r05af_pytest.log" 2>&1
rc=$?; tail -3 "$O/r05af_pytest.log"; [ $rc -eq 0 ] || exit $rc
run() {  # tag, lib dir or "tree", command...
  local tag="$1" lib="$2"; shift 2
  local pre=""; [ "$lib" != tree ] && pre="tools/ab_run.py --lib-dir $lib"
  timeout -k 10 300 python -u $pre "$@" > "$O/r05af_$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$O/r05af_$tag.log"; exit 1; }
  echo "$tag $(grep '^{' "$O/r05af_$tag.log" | tail -1 | cut -c1-520)"
}
for rep in 0 1 2; do
  run vit_tree_$rep tree tools/vit_bench.py
  run vit_w0_$rep ab_gemm/w0 tools/vit_bench.py
done
cd /tmp && export TMPDIR=/tmp
for arm in tree w0; do
  pre=""; [ $arm != tree ] && pre="$R/tools/ab_run.py --lib-dir $R/ab_gemm/w0"
  timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
      --output-format csv -d /tmp/pmc_af_$arm/pass1 -o run -- python3 $pre "$R/tools/vit_bench.py" --iters 1 > "$O/r05af_pmc_$arm.log" 2>&1 \
      || { echo "pmc $arm failed"; tail -3 "$O/r05af_pmc_$arm.log"; exit 1; }
  python3 "$R/tools/pmc_summary.py" /tmp/pmc_af_$arm Split > "$O/r05af_pmc_$arm.txt" 2>&1
  echo "== $arm"; grep -v "^    " "$O/r05af_pmc_$arm.txt" | cut -c1-330
done
