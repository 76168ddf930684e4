"""Build libfibinet_hip.so in-tree with hipcc for gfx950 (no CUDA, no torch extension API).

``python -m ctr_recommendation_amd.build`` or ``__graft_entry__.build()``.  Objects are
compiled in parallel and cached by source mtime under ``build/``; the shared library lands
next to this file so it travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

from . import gen_thunks

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ROOT = os.path.dirname(HERE)
BUILD = os.path.join(ROOT, "build", "fibinet_hip")
LIB = os.path.join(HERE, "libfibinet_hip.so")
SOURCES = ["capi.cpp", "gemm.hip", "fields.hip", "mlp.hip", "optim.hip", "exchange.hip", "collate.hip", "bilinear.hip", "plan.cpp", "comm.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result",
         "-I", CSRC, "-I", os.path.join(ROOT, "include")]


def _compile(src: str, build_dir: str = BUILD, defines=()) -> str:
    path = os.path.join(CSRC, src)
    obj = os.path.join(build_dir, src + ".o")
    deps = [path] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith((".h", ".inc"))]
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return obj
    cmd = [HIPCC] + FLAGS + [f"-D{d}" for d in defines] + ["-c", path, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC, "-O3", "-fPIC", "-std=c++17", "-I", CSRC, "-I", os.path.join(ROOT, "include"), "-c", path,
               "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr}")
    return obj


def build(verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    gen_thunks.write_if_changed(verbose)     # the step programs' thunks follow include/fibinet.h
    with ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        objs = list(ex.map(_compile, SOURCES))
    newest = max(os.path.getmtime(o) for o in objs)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < newest:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs + ["-ldl"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


# A/B builds of the library (never the product): name -> preprocessor defines.  Built into
# tools/variants/libfibinet_hip_<name>.so and selected with FBN_LIB_PATH (_lib.py).
VARIANTS = {
    # table and dense Adam with correctly rounded sqrt / division, unfused (parity bisection)
    "ieee": ("FBN_ADAM_IEEE",),
    # the replay engine's constants one step at a time (round 4's form; A/B of FBN_REPLAY_BLOCK4)
    "rstep1": ("FBN_REPLAY_BLOCK4=0",),
    # the main-stream step kernels at wave priority 3 instead of 2 (A/B of FBN_MAIN_PRIO_LEVEL)
    "prio3": ("FBN_MAIN_PRIO_LEVEL=3",),
}


def build_variant(name: str, verbose: bool = True) -> str:
    defines = VARIANTS[name]
    bdir = os.path.join(ROOT, "build", "variant_" + name)
    gen_thunks.write_if_changed(verbose)
    os.makedirs(bdir, exist_ok=True)
    with ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        objs = list(ex.map(lambda s: _compile(s, bdir, defines), SOURCES))
    out = os.path.join(ROOT, "tools", "variants", f"libfibinet_hip_{name}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(o) for o in objs):
        r = subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs + ["-ldl"],
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print(f"built {out}")
    return out


if __name__ == "__main__":
    if len(sys.argv) > 1:
        for v in sys.argv[1:]:
            build_variant(v)
        sys.exit(0)
    build()
    sys.exit(0)
