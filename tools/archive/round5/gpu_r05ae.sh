#!/bin/bash
# Round-5 GPU batch ae: FFN epilogue writes as paired b128 (tree, MLG_FFN_STAGE_W) vs per-half b64
# (ab_ffn/w0): LightGlue / LoFTR / kernel GPU tests, LightGlue stage bench + LoFTR bench ABAB (digests),
# then a PMC pass per arm for the FFN's LDS conflict share.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_lightglue_gpu.py tests/test_superglue_gpu.py tests/test_loftr_gpu.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > "$O/r05ae_pytest.log" 2>&1
rc=$?; tail -3 "$O/r05ae_pytest.log"; [ $rc -eq 0 ] || exit $rc
run() {  # tag, lib dir or "tree", command...
  local tag="$1" lib="$2"; shift 2
  local pre=""; [ "$lib" != tree ] && pre="tools/ab_run.py --lib-dir $lib"
  timeout -k 10 300 python -u $pre "$@" > "$O/r05ae_$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$O/r05ae_$tag.log"; exit 1; }
  echo "$tag $(grep '^{' "$O/r05ae_$tag.log" | tail -1 | cut -c1-520)"
}
for rep in 0 1; do
  run lg_tree_$rep tree tools/lg_bench.py --pairs 2048 --iters 2
  run lg_w0_$rep ab_ffn/w0 tools/lg_bench.py --pairs 2048 --iters 2
done
run lf_tree tree tools/loftr_bench.py --frames 64 --pairs 64
run lf_w0 ab_ffn/w0 tools/loftr_bench.py --frames 64 --pairs 64
cd /tmp && export TMPDIR=/tmp
for arm in tree w0; do
  pre=""; [ $arm != tree ] && pre="$R/tools/ab_run.py --lib-dir $R/ab_ffn/w0"
  timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
      --output-format csv -d /tmp/pmc_ae_$arm/pass1 -o run -- python3 $pre "$R/tools/lg_bench.py" --pairs 512 --iters 1 > "$O/r05ae_pmc_$arm.log" 2>&1 \
      || { echo "pmc $arm failed"; tail -3 "$O/r05ae_pmc_$arm.log"; exit 1; }
  python3 "$R/tools/pmc_summary.py" /tmp/pmc_ae_$arm k_lg_ffn > "$O/r05ae_pmc_$arm.txt" 2>&1
  echo "== $arm"; cut -c1-330 "$O/r05ae_pmc_$arm.txt"
done
