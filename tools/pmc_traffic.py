"""Per-kernel HBM bytes per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

    python tools/pmc_traffic.py <pass-dir-root> <out.json>

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  gfx950 correction
(MI355X_MICROARCH.md, HBM / rocprofv3): FETCH_SIZE reports half the bytes of wide
coalesced streaming reads, so fetched bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is
exact.  Infinity-Cache hits are counted (not excluded).  Keyed by bench.py's slot
names for the kernels that map one-to-one onto a slot.
"""
import collections
import csv
import glob
import json
import os
import sys

SLOT_KERNELS = {"lightglue_attention": "k_attention_varlen", "lightglue_ffn_fused": "k_lg_ffn",
                "lightglue_qkv_gemms": "k_lg_proj", "vit_attention": "k_attention(",
                "superpoint_conv3x3": "k_conv3x3"}


def main():
    root, out = sys.argv[1], sys.argv[2]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(root + "/pass*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for slot, pat in SLOT_KERNELS.items():
        fetch, write = [], []
        for name, d in vals.items():
            key = name.replace("(anonymous namespace)::", "")
            if pat in key:
                fetch += d.get("FETCH_SIZE", [])
                write += d.get("WRITE_SIZE", [])
        if not fetch or not write:
            continue
        pairs = int(os.environ.get("PAIRS", "4096"))
        fb = 2.0 * 1024 * sum(fetch) / len(fetch)
        wb = 1024.0 * sum(write) / len(write)
        res[slot] = {"kernel": pat.rstrip("("), "dispatches": len(fetch), "pairs": pairs,
                     "fetch_bytes_per_launch": round(fb),
                     "write_bytes_per_launch": round(wb), "bytes_per_launch": round(fb + wb),
                     "source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate runs) of "
                               f"tools/lg_bench.py --iters 1 --pairs {pairs} (one {pairs}-pair LightGlue call = "
                               "bench.py's lg_chunk); FETCH_SIZE x2 (gfx950)"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
