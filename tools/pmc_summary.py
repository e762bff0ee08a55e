"""Summarise rocprofv3 --pmc pass directories per kernel (averages per dispatch), with the
derived utilisations (gfx950 units, MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES counts
cycles summed over SIMDs, GRBM_GUI_ACTIVE sums the 8 XCDs' cycles).

    python tools/pmc_summary.py gpurun_out/pmc_x_lg [name-filter ...]

mfma_util  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
valu_per_mfma, trans_share = SQ_INSTS_VALU_TRANS_F32 / SQ_INSTS_VALU,
coexec_share = SQ_VALU_MFMA_COEXEC_CYCLES / SQ_VALU_MFMA_BUSY_CYCLES (VALU issued while
the MFMA pipe is busy), lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS,
wait_share = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES.
"""
import collections
import csv
import glob
import json
import sys

SIMDS = 1024  # 256 CUs x 4


def short(name):
    """'void (anonymous namespace)::k_lg_ffn<false, 64, 4>(unsigned short const*, ...)' ->
    'k_lg_ffn<false, 64, 4>' (template arguments kept, parameter list dropped)."""
    name = name.replace("(anonymous namespace)::", "").strip()
    if name.startswith("void "):
        name = name[5:]
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0 and i > 0:
            return name[:i]
    return name


def load(root):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(root + "/pass*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} | {"_dispatches": max(len(v) for v in d.values())}
            for k, d in agg.items()}


def derived(a):
    out = {}
    g = a.get("GRBM_GUI_ACTIVE", 0)
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in a:
        out["mfma_util"] = round(a["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * SIMDS), 4)
        out["kernel_us_at_2.4GHz"] = round(g / 8 / 2400, 1)
    if a.get("SQ_INSTS_MFMA"):
        out["valu_per_mfma"] = round(a.get("SQ_INSTS_VALU", 0) / a["SQ_INSTS_MFMA"], 2)
    if a.get("SQ_INSTS_VALU"):
        out["trans_share"] = round(a.get("SQ_INSTS_VALU_TRANS_F32", 0) / a["SQ_INSTS_VALU"], 3)
    if a.get("SQ_VALU_MFMA_BUSY_CYCLES"):
        out["coexec_share"] = round(a.get("SQ_VALU_MFMA_COEXEC_CYCLES", 0) / a["SQ_VALU_MFMA_BUSY_CYCLES"], 3)
    if a.get("SQ_ACTIVE_INST_LDS"):
        out["lds_conflict"] = round(a.get("SQ_LDS_BANK_CONFLICT", 0) / a["SQ_ACTIVE_INST_LDS"], 3)
    if a.get("SQ_WAVE_CYCLES"):
        out["wait_share"] = round(a.get("SQ_WAIT_INST_ANY", 0) / a["SQ_WAVE_CYCLES"], 3)
    return out


def main():
    root, filters = sys.argv[1], sys.argv[2:]
    data = load(root)
    rows = sorted(data.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0) * kv[1]["_dispatches"])
    for name, a in rows:
        if filters and not any(x in name for x in filters):
            continue
        if not a.get("SQ_INSTS_VALU") and not a.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            continue
        print(name, json.dumps(derived(a)))
        print("   ", json.dumps({k: round(v, 1) for k, v in sorted(a.items())}))


if __name__ == "__main__":
    main()
