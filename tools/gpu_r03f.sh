#!/bin/bash
# FFN co-scheduling A/B: in-tree build vs lg_ffn compiled -fno-slp-vectorize / with MFMA
# wait-state padding / both (tools/ffn_variants.sh)
mkdir -p gpurun_out
timeout -k 10 150 python -u tools/ffn_interference.py --victims ffn --partners attn,proj --repeats 12 --analyse > gpurun_out/r03f_ctl.log 2>&1 || exit 1
for v in slp pad both; do
  timeout -k 10 150 python -u tools/ab_run.py --lib-dir ab_ffn_$v tools/ffn_interference.py --victims ffn --partners attn,proj --repeats 12 > gpurun_out/r03f_$v.log 2>&1 || exit 1
done
for f in ctl slp pad both; do echo "== $f"; grep summary gpurun_out/r03f_$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['summary']['ffn']; print({k: (v['runs_differing'], v['max_tiles_differing']) for k, v in d.items()})"; done
