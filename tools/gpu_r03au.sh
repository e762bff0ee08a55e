#!/bin/bash
# r03au: final HEAD: full GPU suite, smoke, bench default (5120 pairs per call, traffic from the 5120-pair PMC file)
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r03au_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03au_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03au_smoke.log 2>&1 || { tail -5 gpurun_out/r03au_smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/r03au_bench.json 2> gpurun_out/r03au_bench.err || { tail -5 gpurun_out/r03au_bench.err; exit 1; }
python3 -c "import json; l=json.loads(open('gpurun_out/r03au_bench.json').read().strip().splitlines()[-1]); r=l['roofline']; print(l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections']['total'], r['frac'], r['avg_launch_us'], r['traffic'], l['cpu_baseline']['value'])"
