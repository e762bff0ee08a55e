#!/bin/bash
# r03j: LoFTR implicit-GEMM backbone + chunked linear attention / dual softmax: tests, timing, profile, bench line
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_loftr_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r03j_loftr_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03j_loftr_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/loftr_bench.py --frames 32 --pairs 32 > gpurun_out/r03j_loftr.json 2>&1 || exit 1
tail -1 gpurun_out/r03j_loftr.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_loftr_j -o loftr -- python3 tools/loftr_bench.py --frames 32 --pairs 32 > gpurun_out/r03j_prof.log 2>&1 || { tail -5 gpurun_out/r03j_prof.log; exit 1; }
timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r03j_bench.json 2> gpurun_out/r03j_bench.err || { tail -5 gpurun_out/r03j_bench.err; exit 1; }
python3 -c "import json; l=json.loads(open('gpurun_out/r03j_bench.json').read().strip().splitlines()[-1]); print(l['value'], json.dumps(l.get('loftr')))"
