"""Build-level guards (CPU only: hipcc cross-compiles gfx950 without a GPU).

Every HIP kernel must run from registers: a runtime-indexed register array silently becomes
scratch (private memory) and slowed pairs_bwd 4x once.  Compile each source with the
resource-usage remarks and fail on any kernel with a non-zero ScratchSize.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ctr_recommendation_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src", sorted(f for f in os.listdir(CSRC) if f.endswith(".hip")))
def test_no_kernel_uses_scratch(src, tmp_path):
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", os.path.join(CSRC, src),
                        "-o", str(tmp_path / "k.o"), "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    names = re.findall(r"Function Name: (\S+)", r.stderr)
    scratch = [int(x) for x in re.findall(r"ScratchSize \[bytes/lane\]: (\d+)", r.stderr)]
    assert names and len(names) == len(scratch)
    bad = [(n, s) for n, s in zip(names, scratch) if s]
    assert not bad, f"kernels using scratch: {bad}"
