#!/bin/bash
# PMC passes (one rocprofv3 run each, never combined with tracing) over tools/proj_ab.py:
# the LightGlue projection / FFN kernels and the generic GEMM at the same shapes.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc_proj_${1:-x}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
            "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d "$OUT/pass$i" -o run -- \
      python3 "$REPO/tools/proj_ab.py" --iters 1 --tokens 524288 > "$OUT/pass$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pass$i.log"; exit $rc; fi
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/pass*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(unsigned")[0].replace("(anonymous namespace)::", "")[-60:]
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        agg[name]["_n_" + r["Counter_Name"]] += 1
for name in sorted(agg, key=lambda n: -agg[n].get("SQ_BUSY_CYCLES", 0))[:10]:
    d = agg[name]
    print(name, {k: round(v / max(d.get("_n_" + k, 1), 1), 1) for k, v in d.items() if not k.startswith("_n_")})
PY
