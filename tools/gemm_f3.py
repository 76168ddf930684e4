"""The MLP's first GEMM (C3: 8192 x 512 x 1920, bf16) timed the ways the product runs it, on one box,
interleaved rounds (tuning aid):

  plain      fbn_gemm, no bias / statistics
  bias+stats fbn_gemm with the bias and the fused BatchNorm tile statistics
  trainer    fbn_gemm_split as ops.forward calls it: A = [Vc16 | pair block of c], bias, statistics
  torch      torch.mm (hipBLASLt) on the same bf16 operands, f32 output
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ctr_recommendation_amd import ops

dev = "cuda"
M, N, K, d = 8192, 512, 1920, 128
bf = torch.bfloat16
A = torch.randn((M, K), device=dev).to(bf)
Vc16 = A[:, :5 * d].contiguous()
c = A.clone()                      # the pair block is read from columns 5d.. of c
W = torch.randn((N, K), device=dev).to(bf)
bias = torch.randn(N, device=dev)
C = torch.empty((M, N), device=dev)
tiles = torch.empty(((M + 63) // 64, N, 2), device=dev)
st = ops._lib.stream_handle()


def plain():
    ops.gemm(A, W, C, M, N, K, K, K, N, False, True, bf16=True, stream=st)


def bias_stats():
    ops.gemm(A, W, C, M, N, K, K, K, N, False, True, bias=bias, bf16=True, stream=st, stats=tiles)


def trainer():
    ops.gemm_split(Vc16, W, C, M, N, K, 5 * d, K, N, False, True, bias=bias, stream=st, stats=tiles,
                   A2=c[:, 5 * d:], lda2=K, kseg=5 * d)


def lib():
    torch.mm(A, W.T, out_dtype=torch.float32)


def main():
    arms = {"plain": plain, "bias+stats": bias_stats, "trainer": trainer, "torch": lib}
    res = {k: [] for k in arms}
    for _ in range(4):
        for name, fn in arms.items():
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(1_000_000)
            e0.record()
            for _ in range(30):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / 30 * 1e3)
    ref = (A.float() @ W.float().T) + bias
    trainer()
    torch.cuda.synchronize()
    err = ((C - ref).abs().max() / ref.abs().max()).item()
    for name, v in res.items():
        v = sorted(v)
        print(f"F3 {name:11s} median {v[len(v) // 2]:6.2f} us  min {v[0]:6.2f} us  ({2 * M * N * K / v[0] / 1e6:5.0f} TF)")
    print(f"trainer form rel err {err:.1e}")


if __name__ == "__main__":
    main()
