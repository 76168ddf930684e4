"""Kernel-level checks of the dense building blocks against plain torch fp32 (pytest -m gpu).

fbn_gemm (MFMA fp32 / bf16, split-K, index remaps) and its fused BatchNorm-statistics
epilogue: per-64-row-tile (sum, M2) from the MFMA epilogue (no split-K) and from the split-K
reduce; C must be bit-identical with and without the statistics.  Tolerances: fp32 GEMM
1e-5 relative to sqrt(K)*|A||B| scale; tile statistics 1e-5 relative.
"""
import pytest
import torch

from ctr_recommendation_amd import ops

pytestmark = pytest.mark.gpu


def _lin(M, N, K, dev, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    A = torch.randn((M, K), generator=g).to(dev)
    W = torch.randn((N, K), generator=g).to(dev) / K ** 0.5
    b = torch.randn((N,), generator=g).to(dev)
    return A, W, b


@pytest.mark.parametrize("M,N,K", [(256, 512, 1920), (200, 256, 1024), (8192, 512, 1920), (8192, 256, 512)])
def test_gemm_fp32_matches_torch(hip_device, M, N, K):
    A, W, b = _lin(M, N, K, hip_device, 1)
    C = torch.empty((M, N), device=hip_device)
    ops.gemm(A, W, C, M, N, K, K, K, N, False, True, bias=b)
    ref = (A.double() @ W.double().T + b.double()).float()
    assert (C - ref).abs().max().item() < 1e-5 * K ** 0.5


@pytest.mark.parametrize("M,N,K,bf16", [(256, 512, 1920, False), (200, 256, 1024, False), (8192, 512, 1920, False),
                                        (8192, 512, 1920, True), (8192, 256, 1024, True), (1000, 256, 512, True)])
def test_gemm_fused_bn_stats(hip_device, M, N, K, bf16):
    A, W, b = _lin(M, N, K, hip_device, 2)
    if bf16:
        A, W = A.bfloat16(), W.bfloat16()
    C0 = torch.empty((M, N), device=hip_device)
    C1 = torch.empty((M, N), device=hip_device)
    nt = (M + 63) // 64
    tiles = torch.full((nt, N, 2), float("nan"), device=hip_device)
    ops.gemm(A, W, C0, M, N, K, K, K, N, False, True, bias=b, bf16=bf16)
    ops.gemm(A, W, C1, M, N, K, K, K, N, False, True, bias=b, bf16=bf16, stats=tiles)
    torch.cuda.synchronize()
    assert torch.equal(C0, C1), "statistics epilogue changed C"
    Cd = C1.double()
    for t in range(nt):
        blk = Cd[t * 64:(t + 1) * 64]
        s = blk.sum(0)
        m2 = ((blk - blk.mean(0)) ** 2).sum(0)
        assert torch.allclose(tiles[t, :, 0].double(), s, rtol=1e-5, atol=1e-4 * blk.shape[0] ** 0.5), t
        assert torch.allclose(tiles[t, :, 1].double(), m2, rtol=1e-5, atol=1e-4), t
    # merged statistics (the BN finalize) == torch's batch statistics
    mean = torch.empty(N, device=hip_device)
    inv = torch.empty(N, device=hip_device)
    ops.bn_train_stats(C1, M, N, mean, inv, None, None, M, ops.NO_COLLECTIVE, ops._lib.stream_handle(C1.device),
                       tiles=tiles)
    var = Cd.var(0, unbiased=False)
    assert torch.allclose(mean.double(), Cd.mean(0), rtol=1e-6, atol=1e-6)
    assert torch.allclose(inv.double(), 1.0 / torch.sqrt(var + ops.BN_EPS), rtol=1e-5)


@pytest.mark.parametrize("transA,transB", [(False, True), (False, False), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(8192, 512, 1920), (200, 136, 256), (512, 1920, 8192), (256, 512, 4096),
                                   (1000, 72, 128), (128, 128, 16384)])
def test_gemm_bf16_all_layouts(hip_device, transA, transB, M, N, K):
    """bf16 operands in every storage layout (the LDS-DMA kernel: K % 64 == 0; ragged M / N
    tiles; the split-K plans of the wgrad shapes) against torch with the same bf16 inputs."""
    g = torch.Generator(device="cpu").manual_seed(3)
    A = torch.randn((K, M) if transA else (M, K), generator=g).to(hip_device).bfloat16()
    Bm = torch.randn((N, K) if transB else (K, N), generator=g).to(hip_device).bfloat16()
    bias = torch.randn((N,), generator=g).to(hip_device)
    C = torch.full((M, N), float("nan"), device=hip_device)
    lda = M if transA else K
    ldb = K if transB else N
    ops.gemm(A, Bm, C, M, N, K, lda, ldb, N, transA, transB, bias=bias)
    a = A.double().T if transA else A.double()
    b = Bm.double().T if transB else Bm.double()
    ref = a @ b + bias.double()
    err = (C.double() - ref).abs().max().item()
    assert err < 2e-5 * K ** 0.5 * 4, err


@pytest.mark.gpu
def test_table_adam_step_vs_ieee(hip_device):
    """The table-row Adam step (v_sqrt_f32 / v_rcp_f32, fused moment updates) that every
    item_emb.weight kernel uses, against the IEEE element step (correctly rounded sqrt and
    division, torch's operation order) on 16M random Adam states (|m| <= sqrt(v)): m within 2 ulp
    of its update's scale, v and p within 8 ulp (p: of max(|p|, |update|)).  The differences come
    from the fused multiply-adds (one rounding where torch has two; under cancellation in
    g*coef + wd*p the fused form is the accurate one) and the ~1 ulp hardware sqrt / rcp."""
    from ctr_recommendation_amd import _lib
    dev = torch.zeros(3, dtype=torch.int64, device=hip_device)
    n = 1 << 22
    for seed in (1, 2, 3, 4):
        _lib.call("fbn_adam_selftest", n, seed, _lib.ptr(dev), _lib.stream_handle(hip_device))
    torch.cuda.synchronize()
    dm, dv, dp = (int(x) / 16 for x in dev.cpu())
    print(f"table Adam step vs IEEE: m {dm} ulp, v {dv} ulp, p {dp} ulp")
    assert dm <= 2.0 and dv <= 8.0, (dm, dv)
    assert dp <= 8.0, dp
