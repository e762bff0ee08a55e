#!/bin/bash
# Round-5 final evidence, final (after the assignment full-tile scans), part B: rocprofv3 kernel-trace stats of a bench run (csv), then the
# attributed PMC passes over the LightGlue stage and the ViT forward (tools/pmc_kernels.sh).
# Only the summaries come back (the raw traces exceed gpurun's 64 MiB return limit).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
P=/tmp/r05zy_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$P" -o run -- \
    python3 -u "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$O/r05zy_prof_bench.json" 2> "$O/r05zy_prof_bench.err"
rc=$?; tail -c 300 "$O/r05zy_prof_bench.json"; [ $rc -eq 0 ] || { tail -5 "$O/r05zy_prof_bench.err"; exit $rc; }
find "$P" -name '*kernel_stats.csv' -exec cp {} "$O/r05zy_rocprof_kernel_stats.csv" \;
ls -la "$O/r05zy_rocprof_kernel_stats.csv"
bash "$R/tools/pmc_kernels.sh" r05zy
for wl in lg vit; do cp "$R/gpurun_out/pmc_r05zy_${wl}.txt" "$O/" 2>/dev/null; rm -rf "$R/gpurun_out/pmc_r05zy_${wl}"; done
du -sh "$O"
