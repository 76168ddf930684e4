"""Run one C3 bf16 GEMM shape ITER times (a target for rocprofv3 --pmc / --kernel-trace passes).

  python tools/gemm_one.py NAME [ITER]      NAME: F3 | F4 | dh1 | dc | U | dWa | dW4
FBN_GEMM_FORCE="bm,bn,split[,waves[,stages]]" forces a plan (see gemm_sweep.py).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ctr_recommendation_amd import ops
from gemm_sweep import SH, operands  # noqa: E402  (tools/ is on sys.path as the script dir)


def main():
    name = sys.argv[1]
    it = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    key = [k for k in SH if k.split()[0] == name][0]
    M, N, K, tA, tB = SH[key]
    A, Bm, lda, ldb, ref = operands(M, N, K, tA, tB)
    C = torch.empty((M, N), device="cuda")
    nb = max(ops._lib.lib().fbn_gemm_workspace_size(M, N, K, 1), 64 * M * N * 4 if M * N < 2 ** 21 else 0)
    ws = torch.empty(nb // 8 + 1, dtype=torch.float64, device="cuda")
    st = ops._lib.stream_handle(C.device)
    for _ in range(it):
        ops.call("fbn_gemm", ops.ptr(A), ops.ptr(Bm), ops.ptr(C), None, M, N, K, lda, ldb, N, int(tA), int(tB),
                 *ops.NO_REMAP, *ops.NO_REMAP, 0.0, 1, 1, 1, None, ops.ptr(ws), nb, st)
    torch.cuda.synchronize()
    err = (C - ref).abs().max().item() / (ref.abs().max().item() + 1e-30)
    print(f"{key} M={M} N={N} K={K} rel err {err:.2e}", flush=True)
    if not err < 1e-3:
        sys.exit(1)


if __name__ == "__main__":
    main()
