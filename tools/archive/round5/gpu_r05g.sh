#!/bin/bash
# Round-5 GPU batch g: LoFTR + isec GPU tests on the three-read dual softmax; A/B
# (digest + time) against the four-read arm (ab_lf_stats0); the bench under rocprofv3
# --kernel-trace --stats for the round's kernel table.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_loftr_gpu.py -m gpu -x -q --timeout 200 \
    --timeout-method thread > "$O/r05g_pytest.log" 2>&1
rc=$?; tail -5 "$O/r05g_pytest.log"; [ $rc -eq 0 ] || exit $rc
tools/gpu_ab.sh ab_lf_stats0 r05g_lf 2 -- tools/loftr_bench.py --frames 64 --pairs 64 > "$O/r05g_lf_ab.txt" 2>&1 || { cat "$O/r05g_lf_ab.txt"; exit 1; }
cat "$O/r05g_lf_ab.txt"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/r05g_prof" -o bench -- python3 -u bench.py --steps 2 --warmup 1 \
    > "$O/r05g_prof_bench.json" 2> "$O/r05g_prof_bench.err" || { tail -5 "$O/r05g_prof_bench.err"; exit 1; }
tail -c 400 "$O/r05g_prof_bench.json"
