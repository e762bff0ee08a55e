#!/bin/bash
# Round-5 GPU batch ab: paired projection staging swizzle r & 7 (tree) vs (r >> 1) & 7 (ab_pp/sw1)
# per the b128 write rule of r05x: kernel + LightGlue GPU tests,
# proj_pipe_check (Q / K / V^T hashes + ms) and the LightGlue stage bench (digest), ABAB;
# then one PMC pass over the stage bench for the projections' LDS conflict share.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_lightglue_gpu.py tests/test_superglue_gpu.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > "$O/r05ab_pytest.log" 2>&1
rc=$?; tail -3 "$O/r05ab_pytest.log"; [ $rc -eq 0 ] || exit $rc
run() {  # tag, lib dir or "tree", command...
  local tag="$1" lib="$2"; shift 2
  local pre=""; [ "$lib" != tree ] && pre="tools/ab_run.py --lib-dir $lib"
  timeout -k 10 300 python -u $pre "$@" > "$O/r05ab_$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$O/r05ab_$tag.log"; exit 1; }
  echo "$tag $(grep '^{' "$O/r05ab_$tag.log" | tail -1 | cut -c1-420)"
}
for rep in 0 1; do
  run pp_tree_$rep tree tools/proj_pipe_check.py --iters 10
  run pp_sw1_$rep ab_pp/sw1 tools/proj_pipe_check.py --iters 10
  run lg_tree_$rep tree tools/lg_bench.py --pairs 2048 --iters 2
  run lg_sw1_$rep ab_pp/sw1 tools/lg_bench.py --pairs 2048 --iters 2
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE \
    --output-format csv -d /tmp/r05ab_lds -o lds -- "$R/tools/bin/lds_probe" > "$O/r05ab_lds.log" 2>&1 || { tail -5 "$O/r05ab_lds.log"; exit 1; }
f=$(find /tmp/r05ab_lds -name '*counter_collection.csv' | head -1); cp "$f" "$O/r05ab_lds_counters.csv"; echo "lds probe ok"
for arm in tree sw1; do
  pre=""; [ $arm != tree ] && pre="$R/tools/ab_run.py --lib-dir $R/ab_pp/sw1"
  timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
      --output-format csv -d /tmp/pmc_ab_$arm/pass1 -o run -- python3 $pre "$R/tools/proj_pipe_check.py" --iters 2 > "$O/r05ab_pmc_$arm.log" 2>&1 \
      || { echo "pmc $arm failed"; tail -3 "$O/r05ab_pmc_$arm.log"; exit 1; }
  python3 "$R/tools/pmc_summary.py" /tmp/pmc_ab_$arm k_lg_proj > "$O/r05ab_pmc_$arm.txt" 2>&1
  head -4 "$O/r05ab_pmc_$arm.txt" | cut -c1-300
done
cd "$R" && timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py tests/test_bench_parity_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > "$O/r05ab_pytest2.log" 2>&1
rc=$?; tail -2 "$O/r05ab_pytest2.log"; exit $rc
