"""Diagnostic build with in-kernel clock stamps (not the product library).

    python tools/clock_probe_build.py OUT_DIR [--src attention.hip] [-D MACRO=V ...]

Copies csrc/ to a scratch directory and stamps thread 0 of every workgroup of the
LightGlue attention tile (k_attention_varlen), the fused FFN (k_lg_ffn) and the
projections (k_lg_proj_res) with s_memtime / s_memrealtime around its work; exports
mlg_probe_clock() (attention), mlg_probe_clock_ffn() and mlg_probe_clock_proj() (median
over the last 16,384 workgroups of d(memtime) / d(memrealtime) x 100 MHz, in GHz) and
links OUT_DIR/libmlgate.so (+ a copy of the tree's libmlgate_torch.so) for
tools/ab_run.py.  Stamps go to arrays of their own that no kernel reads.
The clock the chip holds under an MFMA-dense loop (MI355X_MICROARCH.md 'DVFS give-back'
item 6) is the test of whether saved issue cycles can turn into wall time.
"""
import argparse
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "multi-level-indoor-slam_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall", "-Wno-unused-result", "-fno-slp-vectorize"]
EXTRA = {"attention.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"], "lg_proj.hip": ["-ffp-contract=off"]}  # as the Makefile

def stamp_decl(tag):
    return "\n__device__ ulonglong2 g_clk%s[16384];\n" % tag


def stamp_export(tag, fname):
    return """
extern "C" int %s(double* ghz, int* n) {
    static ulonglong2 h[16384];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_clk%s), sizeof(h)) != hipSuccess) return -1;
    static double r[16384];
    int k = 0;
    for (int i = 0; i < 16384; ++i)
        if (h[i].y > 100) r[k++] = (double)h[i].x / (double)h[i].y * 0.1;
    if (!k) return -2;
    std::sort(r, r + k);
    *ghz = r[k / 2];
    *n = k;
    return 0;
}
""" % (fname, tag)


START = ("    unsigned long long c0__ = 0, r0__ = 0;\n"
         "    if (threadIdx.x == 0) { c0__ = __builtin_amdgcn_s_memtime(); r0__ = __builtin_amdgcn_s_memrealtime(); }\n")


def end(tag):
    return ("    if (threadIdx.x == 0) {\n"
            "        const unsigned long long c1__ = __builtin_amdgcn_s_memtime(), r1__ = __builtin_amdgcn_s_memrealtime();\n"
            "        g_clk%s[blockIdx.x & 16383] = make_ulonglong2(c1__ - c0__, r1__ - r0__);\n"
            "    }\n" % tag)


# file -> (tag, exported name, start anchor (stamp goes before it), end anchor (stamp goes
# before its last line, the kernel's closing brace))
KERNELS = {
    "attention.hip": ("", "mlg_probe_clock",
                      "    attention_tile_pipe(smem, Q + ((size_t)h * Npad + tk.x) * 64",
                      "                        ldo);\n}\n"),
    "lg_ffn.hip": ("_ffn", "mlg_probe_clock_ffn",
                   "    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, col = lane & 31, hh = lane >> 5;\n"
                   "    for (int i = tid; i < 512; i += NTH) {",
                   "        __syncthreads();  // the next tile overwrites the LDS image\n    }\n}\n"),
    "lg_proj.hip": ("_proj", "mlg_probe_clock_proj",
                    "    constexpr int N = SELF ? 768 : 512, NPART = SELF ? 3 : 2, R = 64;",
                    "        if (tn >= ntiles) break;\n        t = tn;\n    }\n}\n"),
}


def patch(fname, src):
    tag, export, a0, a1 = KERNELS[fname]
    assert src.count(a0) == 1, (fname, "start anchor")
    assert src.count(a1) == 1, (fname, "end anchor")
    src = src.replace(a0, START + a0, 1)
    src = src.replace(a1, a1[:-2] + end(tag) + "}\n", 1)
    src = src.replace("namespace {\n", stamp_decl(tag) + "namespace {\n", 1)
    return "#include <algorithm>\n" + src + stamp_export(tag, export)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out_dir")
    ap.add_argument("--src", default=None, help="attention.hip variant to stamp instead of the tree's")
    ap.add_argument("-D", action="append", default=[])
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="clk_")
    work = os.path.join(tmp, "csrc")
    shutil.copytree(CSRC, work, symlinks=True)
    for fname in KERNELS:
        srcpath = a.src if (fname == "attention.hip" and a.src) else os.path.join(CSRC, fname)
        with open(srcpath) as f:
            src = patch(fname, f.read())
        with open(os.path.join(work, fname), "w") as f:
            f.write(src)
        extra = EXTRA.get(fname, [])
        obj = os.path.join(work, "build", fname + ".o")
        subprocess.check_call([HIPCC] + FLAGS + extra + ["-D" + d for d in a.D] + ["-c", fname, "-o", obj], cwd=work)
    os.makedirs(a.out_dir, exist_ok=True)
    objs = sorted(os.path.join(work, "build", o) for o in os.listdir(os.path.join(work, "build")) if o.endswith(".o"))
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-o", os.path.join(a.out_dir, "libmlgate.so")]
                          + objs + ["-lz", "-lpthread"])
    shutil.copy(os.path.join(ROOT, "multi-level-indoor-slam_amd", "mlgate", "libmlgate_torch.so"), a.out_dir)
    shutil.rmtree(tmp)


if __name__ == "__main__":
    main()
