"""Build variants of libfibinet_hip.so with extra -D flags (tuning only).

  python tools/variants.py NAME "-DFOO=1 -DBAR=2" [NAME2 "..."]
Libraries land in tools/variants/lib_NAME.so (git-ignored; they travel to the GPU box with the
snapshot); select one with FBN_LIB_PATH=tools/variants/lib_NAME.so.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ctr_recommendation_amd import build as B  # noqa: E402

OUT = os.path.join(ROOT, "tools", "variants")


def build_variant(name, flags):
    """flags may contain SRC=<dir> to compile the sources of another tree (e.g. a git worktree)."""
    os.makedirs(OUT, exist_ok=True)
    csrc = B.CSRC
    fl = []
    for f in flags.split():
        if f.startswith("SRC="):
            csrc = f[4:]
        else:
            fl.append(f)
    objs = []
    for src in B.SOURCES:
        obj = os.path.join(OUT, f"{name}_{src}.o")
        cmd = [B.HIPCC] + B.FLAGS + fl + ["-I", csrc, "-c", os.path.join(csrc, src), "-o", obj]
        if src.endswith(".cpp"):
            cmd = [B.HIPCC, "-O3", "-fPIC", "-std=c++17", "-c", os.path.join(csrc, src), "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise SystemExit(r.stderr)
        objs.append(obj)
    lib = os.path.join(OUT, f"lib_{name}.so")
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", lib] + objs, check=True)
    for o in objs:
        os.remove(o)
    print("built", lib)


if __name__ == "__main__":
    args = sys.argv[1:]
    for i in range(0, len(args), 2):
        build_variant(args[i], args[i + 1])
