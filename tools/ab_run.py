"""Same-box A/B of two builds without any switch in the product code: run a script
(bench.py, a tool) with mlgate's native libraries taken from another directory.

    python tools/ab_run.py --lib-dir ab_prefix bench.py --steps 2 --warmup 1

The directory holds a libmlgate.so / libmlgate_torch.so pair built from another
revision (libmlgate_torch.so finds its libmlgate.so through its $ORIGIN rpath).
``use_lib_dir`` is also importable by tools that run both arms in one process
order (it must be called before the first ``_native.lib()`` / ``ops()``)."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-level-indoor-slam_amd"))
sys.path.insert(0, ROOT)


def use_lib_dir(lib_dir):
    from mlgate import _native
    if _native._lib is not None or _native._ops is not None:
        raise RuntimeError("mlgate's libraries are already loaded")
    d = os.path.abspath(lib_dir)
    _native.LIB_PATH = os.path.join(d, "libmlgate.so")
    _native.TORCH_LIB_PATH = os.path.join(d, "libmlgate_torch.so")
    for p in (_native.LIB_PATH, _native.TORCH_LIB_PATH):
        if not os.path.exists(p):
            raise FileNotFoundError(p)


def main():
    args = sys.argv[1:]
    if len(args) < 3 or args[0] != "--lib-dir":
        raise SystemExit(__doc__)
    use_lib_dir(args[1])
    script = args[2]
    sys.argv = [script] + args[3:]
    runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
