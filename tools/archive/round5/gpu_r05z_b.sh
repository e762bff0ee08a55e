#!/bin/bash
# Round-5 final evidence, part B: rocprofv3 kernel-trace stats of a bench run (csv), then the
# attributed PMC passes over the LightGlue stage and the ViT forward (tools/pmc_kernels.sh).
# Only the summaries come back (the raw traces exceed gpurun's 64 MiB return limit).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
P=/tmp/r05z_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$P" -o run -- \
    python3 -u "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$O/r05z_prof_bench.json" 2> "$O/r05z_prof_bench.err"
rc=$?; tail -c 300 "$O/r05z_prof_bench.json"; [ $rc -eq 0 ] || { tail -5 "$O/r05z_prof_bench.err"; exit $rc; }
find "$P" -name '*kernel_stats.csv' -exec cp {} "$O/r05z_rocprof_kernel_stats.csv" \;
ls -la "$O/r05z_rocprof_kernel_stats.csv"
bash "$R/tools/pmc_kernels.sh" r05z
for wl in lg vit; do cp "$R/gpurun_out/pmc_r05z_${wl}.txt" "$O/" 2>/dev/null; rm -rf "$R/gpurun_out/pmc_r05z_${wl}"; done
du -sh "$O"
# the LightGlue attention tile's phase timeline (MLG_ATT_TRACE build ab_attt)
cd "$R"
for cfg in "--n 200 --L 2048 --H 4" "--n 400 --L 1000 --H 4"; do
  timeout -k 10 300 python -u tools/ab_run.py --lib-dir ab_attt tools/attn_trace.py $cfg > "$O/r05z_attn_trace.log" 2>&1 \
    || { tail -5 "$O/r05z_attn_trace.log"; exit 1; }
  grep '^{' "$O/r05z_attn_trace.log" | tee -a "$O/r05z_attn_trace.txt"
done
