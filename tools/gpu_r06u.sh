#!/bin/bash
# Round 6: same-box ABAB of the bench (main stream at high priority, the default) with SuperPoint on its side stream under the ViT
# and the kNN (MLGATE_SP_UNDER_VIT=1) vs SuperPoint after them on the main stream (0).


set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"; T="${1:-r06u}"
mkdir -p "$O"
cd "$R"
for k in 0 1; do
  for pr in 0 1; do
    MLGATE_SP_UNDER_VIT=$pr timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ingest \
        --loftr-pairs 0 > "$O/${T}_p${pr}_$k.json" 2> "$O/${T}_p${pr}_$k.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$O/${T}_p${pr}_$k.err"; exit $rc; }
    python - "$O/${T}_p${pr}_$k.json" $pr <<'PY'
import json, sys
l = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print(json.dumps({"sp_under_vit": int(sys.argv[2]), "value": l["value"], "ms_per_step": l["ms_per_step"], "frac": l["roofline"]["frac"],
                  "attn_us": l["roofline"]["avg_launch_us"], "rej": l["config"]["false_loop_closure_rejections"]["total"]}))
PY
  done
done
