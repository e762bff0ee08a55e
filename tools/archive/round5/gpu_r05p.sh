#!/bin/bash
# Round-5 GPU batch p: SuperPoint of the keyframes past the first LightGlue chunk on a side
# stream (MLGATE_SP_OVERLAP=1, default) vs all up front (=0): pipeline GPU tests, then the
# bench ABAB on one box (rejection counts must agree).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py tests/test_distributed_gpu.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > "$O/r05p_pytest.log" 2>&1
rc=$?; tail -3 "$O/r05p_pytest.log"; [ $rc -eq 0 ] || exit $rc
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --loftr-pairs 0"
for rep in 0 1; do
  for ov in 1 0; do
    MLGATE_SP_OVERLAP=$ov timeout -k 10 300 python -u $B > "$O/r05p_bench_ov${ov}_$rep.json" 2> "$O/r05p_bench_ov${ov}_$rep.err" \
      || { echo "bench ov=$ov failed"; tail -5 "$O/r05p_bench_ov${ov}_$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['false_loop_closure_rejections'])" "$O/r05p_bench_ov${ov}_$rep.json" "ov=$ov rep=$rep"
  done
done
