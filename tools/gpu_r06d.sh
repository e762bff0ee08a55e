#!/bin/bash
# Round 6 evidence (interim): the default bench line, rocprofv3 kernel stats of a bench run,
# the attributed PMC passes (LightGlue stage, ViT forward), and the printed measurements of
# the N = 19,163 gate and LoFTR split-vs-exact tests.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"; T="${1:-r06d}"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u bench.py > "$O/${T}_bench.json" 2> "$O/${T}_bench.err"
rc=$?; tail -c 300 "$O/${T}_bench.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_scale_gpu.py tests/test_loftr_gpu.py -k "orbslam3 or exact_arm" -s -q \
    --timeout 300 --timeout-method thread > "$O/${T}_prints.log" 2>&1
rc=$?; grep -E "shared|lg_chunk|passed|failed" "$O/${T}_prints.log"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
P=/tmp/${T}_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$P" -o run -- \
    python3 -u "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --loftr-pairs 0 > "$O/${T}_prof_bench.json" 2> "$O/${T}_prof_bench.err"
rc=$?; tail -c 300 "$O/${T}_prof_bench.json"; [ $rc -eq 0 ] || { tail -5 "$O/${T}_prof_bench.err"; exit $rc; }
find "$P" -name '*kernel_stats.csv' -exec cp {} "$O/${T}_rocprof_kernel_stats.csv" \;
bash "$R/tools/pmc_kernels.sh" "$T"
for wl in lg vit; do rm -rf "$R/gpurun_out/pmc_${T}_${wl}"; done
du -sh "$O"
