"""Diagnostic build of the attention tile with in-kernel clock stamps (not the product).

    python tools/clock_probe_build.py OUT_DIR [--src attention.hip] [-D MACRO=V ...]

Copies csrc/ to a scratch directory, stamps thread 0 of every k_attention_varlen
workgroup with s_memtime / s_memrealtime around its tile, adds mlg_probe_clock()
(median over workgroups of d(memtime) / d(memrealtime) x 100 MHz, in GHz) and links
OUT_DIR/libmlgate.so (+ a copy of the tree's libmlgate_torch.so) for tools/ab_run.py.
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
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall", "-Wno-unused-result", "-fno-slp-vectorize",
         "-mllvm", "-amdgpu-mfma-vgpr-form"]

STAMP_DECL = """
__device__ ulonglong2 g_clk[16384];
"""
STAMP_EXPORT = """
extern "C" int mlg_probe_clock(double* ghz, int* n) {
    static ulonglong2 h[16384];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_clk), sizeof(h)) != hipSuccess) return -1;
    double r[16384];
    int k = 0;
    for (int i = 0; i < 16384; ++i)
        if (h[i].y > 100) r[k++] = (double)h[i].x / (double)h[i].y * 0.1;
    if (!k) return -2;
    std::sort(r, r + k);
    *ghz = r[k / 2];
    *n = k;
    return 0;
}
"""


def patch(src):
    anchor = "    attention_tile_pipe(smem, Q + ((size_t)h * Npad + tk.x) * 64"
    assert anchor in src, "attention tile call not found"
    src = src.replace(anchor, "    unsigned long long c0 = 0, r0 = 0;\n"
                      "    if (threadIdx.x == 0) { c0 = __builtin_amdgcn_s_memtime(); "
                      "r0 = __builtin_amdgcn_s_memrealtime(); }\n" + anchor, 1)
    tail = "                        ldo);\n}\n"
    assert tail in src
    src = src.replace(tail, "                        ldo);\n"
                      "    if (threadIdx.x == 0) {\n"
                      "        const unsigned long long c1 = __builtin_amdgcn_s_memtime(), "
                      "r1 = __builtin_amdgcn_s_memrealtime();\n"
                      "        g_clk[logical & 16383] = make_ulonglong2(c1 - c0, r1 - r0);\n"
                      "    }\n}\n", 1)
    src = src.replace("namespace {\n", STAMP_DECL + "namespace {\n", 1)
    return "#include <algorithm>\n" + src + STAMP_EXPORT


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out_dir")
    ap.add_argument("--src", default=os.path.join(CSRC, "attention.hip"))
    ap.add_argument("-D", action="append", default=[])
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="clk_")
    work = os.path.join(tmp, "csrc")
    shutil.copytree(CSRC, work, symlinks=True)
    with open(a.src) as f:
        src = patch(f.read())
    with open(os.path.join(work, "attention.hip"), "w") as f:
        f.write(src)
    obj = os.path.join(work, "build", "attention.hip.o")
    subprocess.check_call([HIPCC] + FLAGS + ["-D" + d for d in a.D] + ["-c", "attention.hip", "-o", obj], cwd=work)
    os.makedirs(a.out_dir, exist_ok=True)
    objs = sorted(os.path.join(work, "build", o) for o in os.listdir(os.path.join(work, "build")) if o.endswith(".o"))
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-o", os.path.join(a.out_dir, "libmlgate.so")]
                          + objs + ["-lz", "-lpthread"])
    shutil.copy(os.path.join(ROOT, "multi-level-indoor-slam_amd", "mlgate", "libmlgate_torch.so"), a.out_dir)
    shutil.rmtree(tmp)


if __name__ == "__main__":
    main()
