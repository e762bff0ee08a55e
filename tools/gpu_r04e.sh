#!/bin/bash
# r04e: fused split GEMM -- GPU suite (incl. bench-scale parity), bench split vs bf16, FFN hazard arms
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04e_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r04e_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r04e_pytest_gpu.log
for v in split bf16; do
  timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --loftr-pairs 0 --no-ingest --vit $v > gpurun_out/r04e_bench_$v.json 2> gpurun_out/r04e_bench_$v.err || { tail -5 gpurun_out/r04e_bench_$v.err; exit 1; }
  python3 -c "import json; l=json.loads(open('gpurun_out/r04e_bench_$v.json').read().strip().splitlines()[-1]); r=l['roofline']; print('$v', l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections']['total'], {k: v for k, v in r['stage_ms_per_step'].items()})"
done
for arm in ctl slp slpwait slpnont; do
  timeout -k 10 300 python -u tools/ab_run.py --lib-dir ab_ffn_$arm tools/ffn_interference.py --victims ffn --partners attn,proj --repeats 12 > gpurun_out/r04e_ffn_$arm.log 2>&1 || { tail -5 gpurun_out/r04e_ffn_$arm.log; exit 1; }
  echo "$arm $(tail -1 gpurun_out/r04e_ffn_$arm.log)"
done
