#!/bin/bash
# Same-box sweep of the LightGlue chunk size (pairs per mlg_lightglue call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CHUNKS:-2048 1024 4096 1024}; do
  timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --lg-chunk $c > gpurun_out/chunk_$c.log 2>&1
  rc=$?; echo "chunk=$c rc=$rc"; tail -1 gpurun_out/chunk_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['stage_ms_per_step']['lightglue_attention'], d['config']['false_loop_closure_rejections']['total'])"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/chunk_$c.log; exit $rc; fi
done
