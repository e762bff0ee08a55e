#!/bin/bash
# r03ao: round-3 HEAD evidence (final HEAD (FFN narrow-phase ring 2, build-time knobs)): full GPU suite, smoke, bench,
# rocprof stats, PMC traffic passes of one 4096-pair LightGlue call
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r03ao_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03ao_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ao_smoke.log 2>&1 || { tail -5 gpurun_out/r03ao_smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/r03ao_bench.json 2> gpurun_out/r03ao_bench.err || { tail -5 gpurun_out/r03ao_bench.err; exit 1; }
python3 -c "import json; l=json.loads(open('gpurun_out/r03ao_bench.json').read().strip().splitlines()[-1]); print(l['value'], l['ms_per_step'], l['config']['false_loop_closure_rejections'], l['roofline']['frac'], l['roofline']['avg_launch_us'])"
timeout -k 10 700 bash tools/gpu_profile.sh r03ao || exit 1
timeout -k 10 600 bash tools/pmc_traffic.sh
