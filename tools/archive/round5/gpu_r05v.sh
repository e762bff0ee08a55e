#!/bin/bash
# Round-5 GPU batch v: LoFTR dual softmax over groups of 8 pairs (tree) vs pair by pair
# (ab_lf/g1): LoFTR GPU tests, then loftr_bench digest + time ABAB.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_loftr_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
    > "$O/r05v_pytest.log" 2>&1
rc=$?; tail -3 "$O/r05v_pytest.log"; [ $rc -eq 0 ] || exit $rc
run() {  # tag, lib dir or "tree", command...
  local tag="$1" lib="$2"; shift 2
  local pre=""; [ "$lib" != tree ] && pre="tools/ab_run.py --lib-dir $lib"
  timeout -k 10 300 python -u $pre "$@" > "$O/r05v_$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$O/r05v_$tag.log"; exit 1; }
  echo "$tag $(grep '^{' "$O/r05v_$tag.log" | tail -1 | cut -c1-700)"
}
for rep in 0 1; do
  run lf_tree_$rep tree tools/loftr_bench.py --frames 64 --pairs 64
  run lf_g1_$rep ab_lf/g1 tools/loftr_bench.py --frames 64 --pairs 64
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lf_stats -o run -- \
    python3 "$R/tools/loftr_bench.py" --frames 64 --pairs 64 > "$O/r05v_lf_prof.log" 2>&1 \
    || { echo "loftr prof failed"; tail -3 "$O/r05v_lf_prof.log"; exit 1; }
f=$(find /tmp/lf_stats -name '*kernel_stats.csv' | head -1); cp "$f" "$O/r05v_loftr_kernel_stats.csv"; echo "lf stats copied"
