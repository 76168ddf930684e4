"""Time fbn_gemm on the C3 bf16 shapes under forced tile / split-K plans (tuning aid).

  python tools/gemm_sweep.py [name-filter ...]
FBN_GEMM_FORCE="bm,bn,split" forces a plan; FBN_GEMM_NO_DMA16=1 disables the LDS-DMA NT kernel.
Every timed configuration is also checked against torch (fp32 accumulate of the bf16 operands).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ctr_recommendation_amd import ops

dev = "cuda"
bf = torch.bfloat16
d, B = 128, 8192
KC = 15 * d
SH = {  # name: (M, N, K, transA, transB)
    "F3   c16*Wa^T": (B, 512, KC, False, True),
    "F4   h1*Wb^T": (B, 256, 512, False, True),
    "dh1  dh2*Wb": (B, 512, 256, False, True),
    "dc   dh1*Wa": (B, KC, 512, False, True),
    "U    Vc*W": (5 * B, d, d, False, True),
    "dWa  dh1^T c": (512, KC, B, True, False),
    "dW4  dh2^T h1": (256, 512, B, True, False),
}
PLANS = [None] + [(bm, bn, s) for bm, bn in ((64, 64), (128, 64), (64, 128), (128, 128)) for s in (1, 2, 4, 8)] \
    + [(bm, bn, s, 8, st) for bm, bn in ((128, 128), (128, 64), (64, 128)) for s in (1, 2, 4, 8) for st in (2, 3, 4)]
if os.environ.get("FBN_SWEEP_PLANS"):   # "bm,bn,split[,waves[,stages]];..." replaces the list
    PLANS = [None] + [tuple(int(x) for x in p.split(",")) for p in os.environ["FBN_SWEEP_PLANS"].split(";")]


def operands(M, N, K, tA, tB):
    A = torch.randn((K, M) if tA else (M, K), device=dev).to(bf)
    Bm = torch.randn((N, K) if tB else (K, N), device=dev).to(bf)
    ref = (A.float().T if tA else A.float()) @ (Bm.float().T if tB else Bm.float())
    return A, Bm, (M if tA else K), (K if tB else N), ref


def main():
    only = sys.argv[1:]
    for name, (M, N, K, tA, tB) in SH.items():
        if only and not any(o in name for o in only):
            continue
        A, Bm, lda, ldb, ref = operands(M, N, K, tA, tB)
        C = torch.empty((M, N), device=dev)
        # library reference point: torch.mm (hipBLASLt) on the same bf16 operands, f32 output
        Aop = A.T if tA else A
        Bop = Bm.T if tB else Bm
        try:
            for _ in range(3):
                torch.mm(Aop, Bop, out_dtype=torch.float32)
            lib = lambda: torch.mm(Aop, Bop, out_dtype=torch.float32)
        except (TypeError, RuntimeError):
            lib = lambda: torch.mm(Aop, Bop)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            lib()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"torch {name:15s} M={M:5d} N={N:5d} K={K:5d} {us:6.1f}us ({2 * M * N * K / us / 1e6:5.0f} TF)", flush=True)
        modes = ("old", "dma16") if os.environ.get("FBN_SWEEP_OLD") else ("dma16",)
        for mode in modes:
            if mode == "old":
                os.environ["FBN_GEMM_NO_DMA16"] = "1"
            else:
                os.environ.pop("FBN_GEMM_NO_DMA16", None)
            res = []
            for pl in PLANS:
                if pl is None:
                    os.environ.pop("FBN_GEMM_FORCE", None)
                    split = 1
                else:
                    if K // pl[2] < 64:
                        continue
                    os.environ["FBN_GEMM_FORCE"] = ",".join(str(x) for x in pl)
                    split = pl[2]
                nb = max(ops._lib.lib().fbn_gemm_workspace_size(M, N, K, 1), split * M * N * 4)
                ws = torch.empty(nb // 8 + 1, dtype=torch.float64, device=dev)

                def run():
                    ops.call("fbn_gemm", ops.ptr(A), ops.ptr(Bm), ops.ptr(C), None, M, N, K, lda, ldb, N, int(tA),
                             int(tB), *ops.NO_REMAP, *ops.NO_REMAP, 0.0, 1, 1, 1, None, ops.ptr(ws), nb,
                             ops._lib.stream_handle(C.device))

                C.fill_(float("nan"))
                run()
                torch.cuda.synchronize()
                err = (C - ref).abs().max().item() / (ref.abs().max().item() + 1e-30)
                for _ in range(3):
                    run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    run()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / 20 * 1e3
                res.append((us, pl, err))
            bad = [r for r in res if not (r[2] < 1e-3)]
            res.sort(key=lambda r: r[0])
            if os.environ.get("FBN_SWEEP_ALL"):
                for u, p_, e in res:
                    print(f"    {name:15s} {p_}: {u:.1f}us err {e:.1e}", flush=True)
            dflt = [r for r in res if r[1] is None][0][0]
            fl = 2 * M * N * K
            print(f"{mode:5s} {name:15s} M={M:5d} N={N:5d} K={K:5d} default {dflt:6.1f}us ({fl / dflt / 1e6:5.0f} TF)"
                  f" best: " + "  ".join(f"{p}:{u:.1f}" for u, p, _ in res[:4])
                  + (f"  WRONG: {[(p, e) for _, p, e in bad]}" if bad else ""), flush=True)


if __name__ == "__main__":
    main()
