#!/bin/bash
# Round-5 GPU batch f: the whole GPU suite; A/B of the rotary factor layout (LightGlue
# stage bench) and the split-bf16 LoFTR similarity against ab_base_r05.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$O/r05f_pytest.log" 2>&1
rc=$?; tail -5 "$O/r05f_pytest.log"; [ $rc -eq 0 ] || exit $rc
tools/gpu_ab.sh ab_base_r05 r05f_lg 2 -- tools/lg_bench.py --pairs 2048 --iters 2 > "$O/r05f_lg_ab.txt" 2>&1 || { cat "$O/r05f_lg_ab.txt"; exit 1; }
cat "$O/r05f_lg_ab.txt"
tools/gpu_ab.sh ab_base_r05 r05f_lf 2 -- tools/loftr_bench.py --frames 64 --pairs 64 > "$O/r05f_lf_ab.txt" 2>&1 || { cat "$O/r05f_lf_ab.txt"; exit 1; }
cat "$O/r05f_lf_ab.txt"
timeout -k 10 420 python -u bench.py --steps 3 --warmup 2 > "$O/r05f_bench.json" 2> "$O/r05f_bench.err" || { tail -5 "$O/r05f_bench.err"; exit 1; }
tail -c 1500 "$O/r05f_bench.json"
