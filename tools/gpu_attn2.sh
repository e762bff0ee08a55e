#!/bin/bash
# attention A/B on random operands (online vs fixed shift), then the LightGlue stage bench
set -u
cd "${GRAFT_REPO_ROOT}"
for a in "" "--shifted" "--shifted --qk-std 3"; do
  timeout -k 10 120 python tools/attn_bench.py --pairs 256 --len 2048 $a || exit $?
done
timeout -k 10 300 python tools/lg_bench.py --pairs 1024 --frames 128 || exit $?
