#!/bin/bash
# PMC passes (one rocprofv3 run each, never combined with tracing) over tools/lg_bench.py,
# summarised per kernel for the LightGlue kernels.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc_lg_${1:-x}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
            "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$OUT/pass$i" -o run -- \
      python3 "$REPO/tools/lg_bench.py" --iters 1 > "$OUT/pass$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/pass*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("(anonymous namespace)::", "")[-40:]
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        agg[name]["_n_" + r["Counter_Name"]] += 1
for name in sorted(agg, key=lambda n: -agg[n].get("SQ_BUSY_CYCLES", 0))[:8]:
    d = agg[name]
    print(name, {k: round(v / max(d.get("_n_" + k, 1), 1), 1) for k, v in d.items() if not k.startswith("_n_")})
PY
