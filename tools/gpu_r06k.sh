#!/bin/bash
# Round 6: one-GPU rehearsal of the multi-rank bench flow (MLGATE_BENCH_REHEARSE=1: every
# rank on cuda:0 over gloo) at W = 2 and W = 4 through torch.distributed.run, as the driver
# launches bench.py on a node; timings are meaningless, the line's fields and counts are
# the check (the four-term count must equal the single-rank bench's).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"; T="${1:-r06k}"
mkdir -p "$O"
cd "$R"
export MLGATE_BENCH_REHEARSE=1
for W in 2 4; do
  timeout -k 10 480 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 \
      --master-port $((29520 + W)) bench.py --gpus $W --steps 1 --warmup 1 --lg-chunk 1024 --no-ingest \
      --loftr-pairs 256 > "$O/${T}_w$W.json" 2> "$O/${T}_w$W.err"
  rc=$?; tail -c 600 "$O/${T}_w$W.json"; echo; [ $rc -eq 0 ] || { grep -v amdgpu.ids "$O/${T}_w$W.err" | tail -20; exit $rc; }
done
