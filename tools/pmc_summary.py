"""Summarise rocprofv3 --pmc pass directories per kernel (averages per dispatch).

    python tools/pmc_summary.py gpurun_out/pmc_lg_a [name-filter ...]
"""
import collections
import csv
import glob
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = name.split("(")[0] if not name.startswith("void ") else name[5:].split("(")[0]
    return name[-60:]


def main():
    root, filters = sys.argv[1], sys.argv[2:]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(root + "/pass*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, d in sorted(agg.items(), key=lambda kv: -sum(kv[1].get("SQ_BUSY_CYCLES", [0]))):
        if filters and not any(x in name for x in filters):
            continue
        avg = {k: sum(v) / len(v) for k, v in d.items()}
        print(name, {k: round(v, 1) for k, v in sorted(avg.items())})
        if "SQ_WAVE_CYCLES" in avg and "SQ_BUSY_CYCLES" in avg:
            g = avg.get("GRBM_GUI_ACTIVE", 0)
            print("   mfma_busy/(busy*4)=%.3f  lds_conflict/lds_active=%.3f  wait_any/wave_cycles=%.3f  "
                  "L2 hit=%.3f  fetch MB=%.1f write MB=%.1f  gui_active=%.0f" % (
                      avg.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(avg["SQ_BUSY_CYCLES"] * 4, 1),
                      avg.get("SQ_LDS_BANK_CONFLICT", 0) / max(avg.get("SQ_LDS_IDX_ACTIVE", 1), 1),
                      avg.get("SQ_WAIT_ANY", 0) / max(avg["SQ_WAVE_CYCLES"], 1),
                      avg.get("TCC_HIT_sum", 0) / max(avg.get("TCC_HIT_sum", 0) + avg.get("TCC_MISS_sum", 0), 1),
                      avg.get("FETCH_SIZE", 0) / 1024, avg.get("WRITE_SIZE", 0) / 1024, g))


if __name__ == "__main__":
    main()
