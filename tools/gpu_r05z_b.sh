#!/bin/bash
# Round-5 final evidence, part B: rocprofv3 kernel-trace stats of a bench run (csv), then the
# attributed PMC passes over the LightGlue stage and the ViT forward (tools/pmc_kernels.sh).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/r05z_prof" -o run -- \
    python3 -u "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$O/r05z_prof_bench.json" 2> "$O/r05z_prof_bench.err"
rc=$?; tail -c 300 "$O/r05z_prof_bench.json"; [ $rc -eq 0 ] || { tail -5 "$O/r05z_prof_bench.err"; exit $rc; }
bash "$R/tools/pmc_kernels.sh" r05z
