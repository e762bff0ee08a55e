#!/bin/bash
# Round-5 GPU batch s: projection staging image as whole 128-B lines per 16-lane group
# (tree, MLG_PROJ_STAGE2) vs the row image (ab_proj/s0): kernel + LightGlue GPU tests,
# proj_pipe_check (Q / K / V^T hashes + ms) and the LightGlue stage bench (digest), ABAB;
# then one PMC pass over the stage bench for the projections' LDS conflict share.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_lightglue_gpu.py tests/test_superglue_gpu.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > "$O/r05s_pytest.log" 2>&1
rc=$?; tail -3 "$O/r05s_pytest.log"; [ $rc -eq 0 ] || exit $rc
run() {  # tag, lib dir or "tree", command...
  local tag="$1" lib="$2"; shift 2
  local pre=""; [ "$lib" != tree ] && pre="tools/ab_run.py --lib-dir $lib"
  timeout -k 10 300 python -u $pre "$@" > "$O/r05s_$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$O/r05s_$tag.log"; exit 1; }
  echo "$tag $(grep '^{' "$O/r05s_$tag.log" | tail -1 | cut -c1-420)"
}
for rep in 0 1; do
  run pp_tree_$rep tree tools/proj_pipe_check.py --iters 10
  run pp_s0_$rep ab_proj/s0 tools/proj_pipe_check.py --iters 10
  run lg_tree_$rep tree tools/lg_bench.py --pairs 2048 --iters 2
  run lg_s0_$rep ab_proj/s0 tools/lg_bench.py --pairs 2048 --iters 2
done
cd /tmp && export TMPDIR=/tmp
for arm in tree s0; do
  pre=""; [ $arm != tree ] && pre="$R/tools/ab_run.py --lib-dir $R/ab_proj/$arm"
  timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE \
      --output-format csv -d /tmp/pmc_s_$arm -o run -- python3 $pre "$R/tools/proj_pipe_check.py" --iters 2 > "$O/r05s_pmc_$arm.log" 2>&1 \
      || { echo "pmc $arm failed"; tail -3 "$O/r05s_pmc_$arm.log"; exit 1; }
  python3 "$R/tools/pmc_summary.py" /tmp/pmc_s_$arm k_lg_proj > "$O/r05s_pmc_$arm.txt" 2>&1
  head -4 "$O/r05s_pmc_$arm.txt" | cut -c1-300
done
# LoFTR per-kernel time on the tree (which matching kernels the 0.53 ms per pair is made of)
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lf_stats -o run -- \
    python3 "$R/tools/loftr_bench.py" --frames 64 --pairs 64 > "$O/r05s_lf_prof.log" 2>&1 \
    || { echo "loftr prof failed"; tail -3 "$O/r05s_lf_prof.log"; exit 1; }
f=$(find /tmp/lf_stats -name '*kernel_stats.csv' | head -1); cp "$f" "$O/r05s_loftr_kernel_stats.csv"; echo "lf stats copied"
