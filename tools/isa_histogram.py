"""Instruction histogram of a kernel's hottest loop from hipcc assembly (CPU only).

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form \
        --cuda-device-only -S -o /tmp/attn.s multi-level-indoor-slam_amd/csrc/attention.hip -I include -I multi-level-indoor-slam_amd/csrc
    python tools/isa_histogram.py /tmp/attn.s 'k_attention_varlenILb0ELb0ELi4'

(the flags are the Makefile's rule for attention.hip; use the file's own rule for others.)
Finds the function whose symbol contains the pattern, every backward branch in it (a
loop), and for the loop with the most MFMAs prints the instructions per class: the
per-score softmax work (exp, fma / mul / sub, add, max, cvt / pack), the MFMAs, and the
rest (LDS, memory, moves, wait states, scalar control)."""
import collections
import re
import sys

CLASSES = [
    ("mfma", r"^v_mfma"),
    ("exp (trans)", r"^v_(exp|log|rcp|rsq|sqrt)_"),
    ("fma / mul / sub (f32)", r"^v_(fma|fmac|fmamk|fmaak|mul|sub|subrev)_f32"),
    ("add (f32)", r"^v_add_f32"),
    ("max / min (f32)", r"^v_(max|min|max3|min3)_f32"),
    ("cvt / pack bf16", r"^v_(cvt|perm|pack|pk_)"),
    ("permlane / dpp / swizzle", r"^v_(permlane|mov_b32_dpp|mov_dpp)|_dpp|^ds_swizzle|^ds_bpermute|^ds_permute"),
    ("cndmask / cmp", r"^v_(cndmask|cmp)"),
    ("accvgpr moves", r"^v_accvgpr"),
    ("v_mov", r"^v_mov"),
    ("int / address VALU", r"^v_(add|sub|lshl|lshr|and|or|xor|mad|mul_u|mul_lo|bfe|bfi|lshl_add|add3|lshl_or|and_or|ashr)"),
    ("LDS read", r"^ds_read"),
    ("LDS write", r"^ds_write"),
    ("global / buffer", r"^(global_|buffer_)"),
    ("s_waitcnt", r"^s_waitcnt"),
    ("s_nop", r"^s_nop"),
    ("barrier", r"^s_barrier"),
    ("scalar other", r"^s_"),
]


def function_lines(path, pat):
    lines = open(path).read().split("\n")
    start = None
    for k, ln in enumerate(lines):
        if re.match(r"^_Z\S*:", ln) and pat in ln:
            start = k
            break
    if start is None:
        raise SystemExit(f"no function matching {pat}")
    end = next(k for k in range(start, len(lines)) if lines[k].startswith(".Lfunc_end"))
    return lines[start:end]


def main():
    path, pat = sys.argv[1], sys.argv[2]
    body = function_lines(path, pat)
    labels = {}
    for k, ln in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", ln)
        if m:
            labels[m.group(1)] = k
    loops = []
    for k, ln in enumerate(body):
        m = re.match(r"^\s+s_cbranch_\w+\s+(\.LBB\w+)|^\s+s_branch\s+(\.LBB\w+)", ln)
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] < k:
                loops.append((labels[tgt], k))
    best = None
    for a, b in loops:
        n = sum(1 for ln in body[a:b + 1] if ln.strip().startswith("v_mfma"))
        if best is None or n > best[2]:
            best = (a, b, n)
    a, b, nm = best
    # instructions after a conditional branch up to the next unconditional one are a
    # conditionally executed segment (e.g. the attention tile's lazy O rescale): counted
    # apart, the rest is the path every iteration runs
    hist, cond = collections.Counter(), collections.Counter()
    total = ncond = 0
    in_cond = False
    for ln in body[a:b + 1]:
        t = ln.strip()
        if t.startswith(".LBB"):
            in_cond = False
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        h = cond if in_cond else hist
        if in_cond:
            ncond += 1
        else:
            total += 1
        for name, rx in CLASSES:
            if re.search(rx, op):
                h[name] += 1
                break
        else:
            h["other: " + op] += 1
        if op.startswith("s_cbranch"):
            in_cond = True
        elif op == "s_branch":
            in_cond = False
    nm = hist["mfma"]
    print(f"function ~{pat}: hottest loop = lines {a}..{b}; every-iteration path: {nm} MFMAs, {total} "
          f"instructions; conditional segments: {ncond} instructions ({dict(cond.most_common(4))})")
    for name, _ in CLASSES:
        if hist[name]:
            print(f"  {name:28s} {hist[name]:5d}  {hist[name] / max(nm, 1):6.2f} per MFMA")
    for name in sorted(k for k in hist if k.startswith("other")):
        print(f"  {name:28s} {hist[name]:5d}")
    valu = sum(v for k, v in hist.items() if k not in ("mfma", "LDS read", "LDS write", "global / buffer", "s_waitcnt",
                                                      "s_nop", "barrier", "scalar other") and not k.startswith("other: s_"))
    print(f"  vector ALU (non-MFMA) total    {valu:5d}  {valu / max(nm, 1):6.2f} per MFMA")


if __name__ == "__main__":
    main()
