#!/bin/bash
# Round-6 final evidence, part C: rocprofv3 kernel stats of a bench run, the attributed PMC
# passes (LightGlue stage, ViT forward), and the bench's N = 19,163 stress sub-object.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"; T="${1:-r06z}"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
P=/tmp/${T}_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$P" -o run -- \
    python3 -u "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --loftr-pairs 0 > "$O/${T}_prof_bench.json" 2> "$O/${T}_prof_bench.err"
rc=$?; tail -c 300 "$O/${T}_prof_bench.json"; [ $rc -eq 0 ] || { tail -5 "$O/${T}_prof_bench.err"; exit $rc; }
find "$P" -name '*kernel_stats.csv' -exec cp {} "$O/${T}_rocprof_kernel_stats.csv" \;
bash "$R/tools/pmc_kernels.sh" "$T"
rc=$?; [ $rc -eq 0 ] || exit $rc
for wl in lg vit; do rm -rf "$R/gpurun_out/pmc_${T}_${wl}"; done
cd "$R"
timeout -k 10 500 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ingest --loftr-pairs 0 --stress-keyframes 19163 > "$O/${T}_stress.json" 2> "$O/${T}_stress.err"
rc=$?; tail -c 600 "$O/${T}_stress.json"; du -sh "$O"; exit $rc
