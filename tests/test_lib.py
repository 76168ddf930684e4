"""CPU tests of the C-ABI library and the product/oracle boundary (no GPU compute calls)."""
import ast
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "fibinet.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fbn_[a-z0-9_]+)\s*\(", src)))


def test_library_builds_loads_and_exports_header():
    from ctr_recommendation_amd import _lib
    h = _lib.lib()
    assert h.fbn_version() == 1
    syms = _header_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(h, s), f"{s} declared in include/fibinet.h but not exported"
        assert s in _lib.SIGNATURES, f"{s} has no ctypes signature"
    assert set(_lib.SIGNATURES) == set(syms)


def test_workspace_queries_are_host_only():
    from ctr_recommendation_amd import _lib
    h = _lib.lib()
    assert h.fbn_gemm_workspace_size(16384, 1024, 512, 1) == 0         # enough tiles: no split-K
    assert h.fbn_gemm_workspace_size(512, 1920, 8192, 1) > 0          # wgrad: split-K slabs
    assert h.fbn_fields_bwd_partials_size(128, 3, 11) == 13 * 3 + 6 + 3 * 128 + 11 * 128   # + mm_proj bias partial row
    assert h.fbn_bn_workspace_size(8192, 512) > 0


def test_wgrad_group_split_fills_two_workgroups_per_cu(monkeypatch):
    """The grouped weight-gradient launch's K-slabs (host planning only): by default 3/4 of the
    single launches' slabs, rounded, so C3's four problems (dWa 512 x 1920, dWb 256 x 512, the
    bilinear W 128 x 128 over K = 5B, mm_proj 128 x 128) come to at most two 128 x 128 workgroups
    per CU on 256 CUs; FBN_GROUP_SPLIT_DIV (read per call, fractional allowed) overrides it."""
    from ctr_recommendation_amd import _lib
    h = _lib.lib()
    B = 8192
    probs = [(512, 1920, B), (256, 512, B), (128, 128, 5 * B), (128, 128, B)]
    monkeypatch.delenv("FBN_GROUP_SPLIT_DIV", raising=False)

    def total():
        return sum(((M + 127) // 128) * ((N + 127) // 128) * h.fbn_gemm_slabs_group_split(M, N, K)
                   for M, N, K in probs)
    assert h.fbn_gemm_slabs_split(512, 1920, B) == 8
    assert h.fbn_gemm_slabs_group_split(512, 1920, B) == 6
    assert 384 < total() <= 512
    for M, N, K in probs:
        assert 1 <= h.fbn_gemm_slabs_group_split(M, N, K) <= h.fbn_gemm_slabs_split(M, N, K)
    monkeypatch.setenv("FBN_GROUP_SPLIT_DIV", "2")        # round 3's halving
    assert h.fbn_gemm_slabs_group_split(512, 1920, B) == 4 and total() == 336
    monkeypatch.setenv("FBN_GROUP_SPLIT_DIV", "1")        # fbn_gemm_slabs's own partition
    assert all(h.fbn_gemm_slabs_group_split(M, N, K) == h.fbn_gemm_slabs_split(M, N, K) for M, N, K in probs)


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, "ctr_recommendation_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if not f.endswith(".py"):
                continue
            tree = ast.parse(open(os.path.join(dirpath, f)).read())
            for node in ast.walk(tree):
                if isinstance(node, ast.Import):
                    assert not any(a.name.split(".")[0] == "oracle" for a in node.names), f
                if isinstance(node, ast.ImportFrom):
                    assert (node.module or "").split(".")[0] != "oracle", f


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    from ctr_recommendation_amd import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.lib()


def test_kernels_are_gfx950_code_objects():
    so = os.path.join(ROOT, "ctr_recommendation_amd", "libfibinet_hip.so")
    data = open(so, "rb").read()
    assert b"gfx950" in data


def test_step_program_argument_encoding():
    """Step programs record each call's arguments as 64-bit integer words and doubles and replay it
    through a packed-argument thunk generated from include/fibinet.h (csrc/plan_thunks.inc): an
    int -1 is the word 0xFFFF...F (the thunk casts it back to int), a float the double whose low
    32 bits are its bits.  The committed thunks are what the header generates, every recordable
    SIGNATURES entry has one with the same integer / floating argument counts, and the library
    refuses a recording whose counts differ or that names no entry point."""
    import ctypes
    import struct
    from ctr_recommendation_amd import _lib, gen_thunks
    assert _lib._as_u64(None) == 0
    assert _lib._as_u64(-1) == (1 << 64) - 1
    assert _lib._as_u64(7) == 7
    arr = (ctypes.c_int * 4)()
    assert _lib._as_u64(arr) == ctypes.addressof(arr)
    for x in (1.0, -2.5, 1e-8, 0.999, 3.4e38):
        d = _lib._f32_in_f64(x)
        bits = struct.unpack("<Q", struct.pack("<d", d))[0]
        assert bits >> 32 == 0
        assert struct.unpack("<f", struct.pack("<I", bits))[0] == struct.unpack("<f", struct.pack("<f", x))[0]
    with pytest.raises(TypeError):
        _lib._as_u64(ctypes.byref(ctypes.c_int(0)))
    hdr = open(os.path.join(ROOT, "include", "fibinet.h")).read()
    assert open(gen_thunks.OUT).read() == gen_thunks.generate(hdr), "run python -m ctr_recommendation_amd.gen_thunks"
    thunks = {name: args for name, args in gen_thunks.declarations(hdr)}
    for name, (_, args) in _lib.SIGNATURES.items():
        if name not in thunks:
            continue
        nf = sum(1 for a in args if a in (_lib.F, _lib.D))
        t = thunks[name]
        assert (len(args) - nf, nf) == (sum(1 for a in t if not (a[1] or a[2])), sum(1 for a in t if a[1] or a[2])), name
        assert len(args) - nf <= 48 and nf <= 8, name
    h = _lib.lib()
    prog = _lib.StepProgram("cpu")
    ia, fa = (ctypes.c_ulonglong * 4)(), (ctypes.c_double * 1)()
    assert h.fbn_plan_add_call(ctypes.c_void_p(prog.h), b"fbn_widen_bf16", ia, 4, fa, 0) == 0     # counts match
    assert h.fbn_plan_add_call(ctypes.c_void_p(prog.h), b"fbn_widen_bf16", ia, 3, fa, 0) != 0     # too few
    assert h.fbn_plan_add_call(ctypes.c_void_p(prog.h), b"fbn_no_such_call", ia, 0, fa, 0) != 0
    assert len(prog) == 1
    del prog
    # an empty program runs (host only: no launches)
    prog = _lib.StepProgram("cpu")
    assert len(prog) == 0
    prog.run()
    del prog, h
