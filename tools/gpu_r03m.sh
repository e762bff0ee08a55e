#!/bin/bash
# r03m: attention with the MFMA offset k-step (q in exp2 units from lg_proj): A/B vs ab_base, full GPU suite, bench
mkdir -p gpurun_out
for arm in new base new base; do
  if [ $arm = new ]; then timeout -k 10 200 python -u tools/attn_bench.py --pairs 1024 --len 2048 --iters 5 > gpurun_out/r03m_attn_$arm.json || exit 1
  else timeout -k 10 200 python -u tools/ab_run.py --lib-dir ab_base tools/attn_bench.py --raw-q --pairs 1024 --len 2048 --iters 5 > gpurun_out/r03m_attn_$arm.json || exit 1; fi
  echo $arm $(cat gpurun_out/r03m_attn_$arm.json)
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r03m_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03m_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --no-cpu-baseline --loftr-pairs 0 > gpurun_out/r03m_bench.json 2> gpurun_out/r03m_bench.err || { tail -5 gpurun_out/r03m_bench.err; exit 1; }
python3 -c "import json; l=json.loads(open('gpurun_out/r03m_bench.json').read().strip().splitlines()[-1]); print(l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections'], json.dumps(l['roofline']['stage_ms_per_step']), l['roofline']['frac'], l['roofline']['avg_launch_us'])"
