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
