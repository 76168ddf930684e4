"""Kernel-level checks of the dense building blocks against plain torch fp32 (pytest -m gpu).

fbn_gemm (MFMA fp32 / bf16, split-K, index remaps) and its fused BatchNorm-statistics
epilogue: per-64-row-tile (sum, M2) from the MFMA epilogue (no split-K) and from the split-K
reduce; C must be bit-identical with and without the statistics.  Tolerances: fp32 GEMM
1e-5 relative to sqrt(K)*|A||B| scale; tile statistics 1e-5 relative.
"""
import pytest
import torch

from ctr_recommendation_amd import _lib, ops

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


@pytest.mark.parametrize("transA,transB", [(False, True), (False, False), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(8192, 1920, 512), (512, 1920, 8192), (200, 136, 256), (128, 128, 40960),
                                   (1000, 72, 100)])
def test_gemm_split_bf16x3(hip_device, transA, transB, M, N, K):
    """fbn_gemm bf16 = 2 (split-bf16 x3 over fp32 operands, the bf16_fwd backward's GEMMs) against
    float64: ~2^-16 relative per product (the dropped lo x lo term and the lo rounding), so the
    error bar is 4e-5 x sqrt(K) x |a||b| -- 100x tighter than a plain bf16 GEMM on the same fp32
    inputs (checked beside it), and within 30x of the fp32 MFMA GEMM's."""
    g = torch.Generator(device="cpu").manual_seed(5)
    A = torch.randn((K, M) if transA else (M, K), generator=g).to(hip_device)
    Bm = torch.randn((N, K) if transB else (K, N), generator=g).to(hip_device)
    lda = M if transA else K
    ldb = K if transB else N
    a = A.double().T if transA else A.double()
    b = Bm.double().T if transB else Bm.double()
    ref = a @ b
    errs = {}
    for mode in (2, True, False):
        C = torch.full((M, N), float("nan"), device=hip_device)
        ops.gemm(A, Bm, C, M, N, K, lda, ldb, N, transA, transB, bf16=mode)
        errs[mode] = (C.double() - ref).abs().max().item()
    assert errs[2] < 4e-5 * K ** 0.5, errs
    assert errs[2] * 20 < errs[True], errs            # far better than bf16 operands
    assert errs[2] < 30 * errs[False] + 1e-6, errs    # near fp32


@pytest.mark.parametrize("transA,transB", [(False, True), (False, False), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(8192, 1920, 512), (512, 1920, 8192), (256, 136, 256), (128, 128, 40960)])
def test_gemm_s3_images(hip_device, transA, transB, M, N, K):
    """fbn_gemm_s3 (the bf16_fwd backward's GEMMs): ONE bf16 GEMM over 3 K on the (hi, lo) images
    fbn_convert_bf16 part 2 writes, against float64 -- the same split-bf16 x3 error bar as
    fbn_gemm bf16 = 2 (4e-5 x sqrt(K)); beta = 1 accumulates; and in slab mode (the grouped
    weight-gradient launch, k-major A and B) the sum of its slabs matches the plain launch."""
    g = torch.Generator(device="cpu").manual_seed(7)
    A = torch.randn((K, M) if transA else (M, K), generator=g).to(hip_device)
    Bm = torch.randn((N, K) if transB else (K, N), generator=g).to(hip_device)
    lda = M if transA else K
    ldb = K if transB else N
    a = A.double().T if transA else A.double()
    b = Bm.double().T if transB else Bm.double()
    ref = a @ b
    Ai = torch.empty((2,) + tuple(A.shape), dtype=torch.bfloat16, device=hip_device)
    Bi = torch.empty((2,) + tuple(Bm.shape), dtype=torch.bfloat16, device=hip_device)
    ops.split_images([(A, Ai, A.shape[0], A.shape[1], A.shape[1], 0, ops.NO_REMAP),
                      (Bm, Bi, Bm.shape[0], Bm.shape[1], Bm.shape[1], 0, ops.NO_REMAP)], _lib.stream_handle())
    assert torch.equal(Ai[0], A.bfloat16()) and torch.equal(Ai[1], (A - Ai[0].float()).bfloat16())
    C = torch.full((M, N), float("nan"), device=hip_device)
    ops.gemm_s3(Ai, Bi, C, M, N, K, lda, ldb, N, transA, transB)
    err = (C.double() - ref).abs().max().item()
    assert err < 4e-5 * K ** 0.5, err
    C2 = C.clone()
    ops.gemm_s3(Ai, Bi, C2, M, N, K, lda, ldb, N, transA, transB, beta=1.0)
    assert (C2.double() - 2 * ref).abs().max().item() < 8e-5 * K ** 0.5
    if transA and not transB:
        C3 = torch.full((M, N), float("nan"), device=hip_device)
        sums = ops.DeferredSums()
        assert sums.gemm_slabs(Ai, Bi, C3, M, N, K, lda, ldb, N, True, False, s3=True)
        sums.flush(_lib.stream_handle())
        assert (C3.double() - ref).abs().max().item() < 4e-5 * K ** 0.5


@pytest.mark.parametrize("M,N,K,remap", [(256, 512, 8192, False), (512, 1920, 8192, True), (128, 128, 40960, False),
                                          (16, 16, 20480, False), (128, 128, 8192, False)])
def test_gemm_slabs_deferred_sum(hip_device, M, N, K, remap):
    """The weight-gradient GEMMs' slab mode (fbn_gemm_slabs: split-K slabs left in ws) summed by
    the step's fbn_sum_jobs2 launch beside ordinary column-sum jobs (one with a row stride ld):
    C == torch's op(A) op(B) of the same bf16 operands, written through the mlp.0.weight remap."""
    g = torch.Generator(device="cpu").manual_seed(5)
    A = torch.randn((K, M), generator=g).to(hip_device).bfloat16()      # k-major A (the wgrads' dY)
    Bm = torch.randn((K, N), generator=g).to(hip_device).bfloat16()     # k-major B (activations)
    rc = ops.wa_remap(128) if remap else ops.NO_REMAP
    ldc = 21 * 128 if remap else N
    C = torch.full((M, ldc), float("nan"), device=hip_device)
    part = torch.randn((300, 40), generator=g).to(hip_device)
    out1 = torch.empty(24, device=hip_device)
    out2 = torch.empty(16, device=hip_device)
    sums = ops.DeferredSums()
    assert sums.gemm_slabs(A, Bm, C, M, N, K, M, N, ldc, True, False, rC=rc)
    sums.add(part, 300, 24, out1, ld=40)
    sums.add(part[:, 24:], 300, 16, out2, scale=0.5, ld=40)
    out3 = torch.ones(40, device=hip_device)
    sums.add(part, 300, 40, out3, beta=2.0, ld=40)           # a wide job (16 columns x 16 row streams per block)
    sums.flush(ops._lib.stream_handle(hip_device))
    torch.cuda.synchronize()
    ref = A.double().T @ Bm.double()
    cols = torch.arange(N, device=hip_device)
    if remap:
        cols = cols + torch.where(cols < rc[0], rc[1], rc[2])
    err = (C[:, cols].double() - ref).abs().max().item()
    assert err < 2e-5 * K ** 0.5 * 4, err
    pd = part.double().sum(0)
    assert torch.allclose(out1.double(), pd[:24], rtol=1e-5, atol=1e-4)
    assert torch.allclose(out2.double(), 0.5 * pd[24:], rtol=1e-5, atol=1e-4)
    assert torch.allclose(out3.double(), 2.0 + pd, rtol=1e-5, atol=1e-4)


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


@pytest.mark.gpu
@pytest.mark.parametrize("d,B,dc16", [(128, 8192, 1), (128, 8192, 0), (128, 100, 1), (64, 333, 0), (32, 1000, 1),
                                      (16, 4096, 1), (16, 333, 0)])
def test_fused_bilinear_matches_unfused_math(hip_device, d, B, dc16):
    """fbn_bilinear_fwd / _bwd (one MFMA + pair-product launch each way, U never stored) against
    the same arithmetic in torch on the same bf16 operands: pairs and dU16 within 1 bf16 ulp (U's
    f32 sums may round differently), dV within 2e-5 x max|dV|.  B = 100 / 333: a partial last
    tile of samples.  dc16: the incoming gradient dc in bf16 (fbn_gemm_bf16out's output, the
    trainer's bf16 mode) or f32.  d = 16 (config C2): one wave per 16 samples on the 16x16x16 MFMA."""
    from ctr_recommendation_amd import _lib
    g = torch.Generator(device=hip_device).manual_seed(3)
    V16 = (torch.randn((B, 5, d), generator=g, device=hip_device) * 0.5).to(torch.bfloat16)
    W = torch.randn((d, d), generator=g, device=hip_device) / d ** 0.5
    W16, WT16 = W.to(torch.bfloat16).contiguous(), W.t().contiguous().to(torch.bfloat16)
    KC = 15 * d
    c = torch.zeros((B, KC), dtype=torch.bfloat16, device=hip_device)
    st = _lib.stream_handle(hip_device)
    _lib.call("fbn_bilinear_fwd", _lib.ptr(V16), _lib.ptr(WT16), _lib.ptr(c), B, d, KC, st)
    Vf, Wf = V16.float(), W16.float()
    U = torch.einsum("bfk,kn->bfn", Vf, Wf)
    pairs = [(0, 1), (0, 2), (0, 3), (0, 4), (1, 2), (1, 3), (1, 4), (2, 3), (2, 4), (3, 4)]
    Uabs = torch.einsum("bfk,kn->bfn", Vf.abs(), Wf.abs())          # scale of U's summands
    ref = torch.cat([(Vf[:, i] * U[:, j]) for i, j in pairs], 1).to(torch.bfloat16).float()
    got = c[:, 5 * d:].float()
    # 1 bf16 ulp of the larger value, plus U's f32 summation-order term (U can cancel: its relative
    # error is then not small although its absolute error is)
    slack = torch.cat([(Vf[:, i].abs() * Uabs[:, j]) for i, j in pairs], 1) * 2.0 ** -16
    tol = torch.maximum(ref.abs(), got.abs()) * 2.0 ** -7 + slack
    assert bool(((got - ref).abs() <= tol).all()), ((got - ref).abs() - tol).max().item()
    assert bool((c[:, :5 * d] == 0).all())                       # the V block is not the kernel's
    # backward
    dc = torch.randn((B, KC), generator=g, device=hip_device) * 1e-3
    dc_in = dc.to(torch.bfloat16) if dc16 else dc
    dc = dc_in.float()                                            # the values the kernel sees
    dV = torch.empty((B, 5, d), device=hip_device)
    dU16 = torch.empty((B, 5, d), dtype=torch.bfloat16, device=hip_device)
    _lib.call("fbn_bilinear_bwd", _lib.ptr(dc_in), KC, dc16, _lib.ptr(V16), _lib.ptr(WT16), _lib.ptr(W16),
              _lib.ptr(dV), _lib.ptr(dU16), B, d, st)
    gv = dc[:, :5 * d].view(B, 5, d).clone()
    gu = torch.zeros((B, 5, d), device=hip_device)
    for k, (i, j) in enumerate(pairs):
        gp = dc[:, (5 + k) * d:(6 + k) * d]
        gv[:, i] += gp * U[:, j]
        gu[:, j] += gp * Vf[:, i]
    gu16 = gu.to(torch.bfloat16)
    guabs = torch.zeros_like(gu)
    for k, (i, j) in enumerate(pairs):
        guabs[:, j] += dc[:, (5 + k) * d:(6 + k) * d].abs() * Vf[:, i].abs()
    tol = torch.maximum(gu16.float().abs(), dU16.float().abs()) * 2.0 ** -7 + guabs * 2.0 ** -20
    assert bool(((dU16.float() - gu16.float()).abs() <= tol).all())
    dV_ref = gv + torch.einsum("bfn,kn->bfk", dU16.float(), Wf)
    err = (dV - dV_ref).abs().max().item()
    assert err <= 2e-5 * dV_ref.abs().max().item(), err


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(8192, 1920, 512), (300, 200, 128)])
def test_gemm_bf16out_is_rounded_f32_gemm(hip_device, M, N, K):
    """fbn_gemm_bf16out (the bf16-mode dc = dh1 Wa): the same plan and accumulation as fbn_gemm's
    f32 output, rounded once to bf16 -- bit-identical to the f32 result's round-to-nearest-even."""
    from ctr_recommendation_amd import _lib
    g = torch.Generator(device=hip_device).manual_seed(11)
    A = torch.randn((M, K), generator=g, device=hip_device).to(torch.bfloat16)
    Bt = torch.randn((N, K), generator=g, device=hip_device).to(torch.bfloat16)     # B^T, as WaT
    st = _lib.stream_handle(hip_device)
    C32 = torch.empty((M, N), device=hip_device)
    ops.gemm(A, Bt, C32, M, N, K, K, K, N, False, True, stream=st)
    C16 = torch.empty((M, N), dtype=torch.bfloat16, device=hip_device)
    _lib.call("fbn_gemm_bf16out", _lib.ptr(A), _lib.ptr(Bt), _lib.ptr(C16), M, N, K, K, K, N, 0, 1, st)
    torch.cuda.synchronize()
    assert torch.equal(C16, C32.to(torch.bfloat16))


@pytest.mark.gpu
@pytest.mark.parametrize("d,zipf", [(128, 0.0), (128, 1.05), (16, 1.05), (64, 1.2)])
def test_duplicate_fold_matches_scatter_add(hip_device, d, zipf):
    """fbn_claim_rows + fbn_sparse_fixup_dup (wave sums per claimer, LDS table for popular rows) against
    a float64 scatter-add of every entry's vector: each claimed row's gradient (its claimer's vector,
    plus extra[claimer] when flagged) within 1e-5 of the row's scale; every touched row claimed once.
    Zipf ids: the hottest rows take thousands of entries of a batch."""
    from ctr_recommendation_amd import _lib
    from ctr_recommendation_amd.data import make_device_batches
    B, L, V = 4096, 20, 200_000
    (b, _), = make_device_batches(1, B, V, L, hip_device, seed=5, zipf=zipf)
    n = B * (L + 1)
    st = _lib.stream_handle(hip_device)
    i32 = dict(dtype=torch.int32, device=hip_device)
    map_, slot_row, dup = torch.full((V,), -1, **i32), torch.full((n,), -1, **i32), torch.full((n,), -1, **i32)
    _lib.call("fbn_claim_rows", _lib.ptr(b["item_id"]), _lib.ptr(b["item_seq"]), B, L, V, _lib.ptr(map_),
              _lib.ptr(slot_row), _lib.ptr(dup), None, st)
    g = torch.Generator(device=hip_device).manual_seed(1)
    gvec = torch.randn((B, 2, d), generator=g, device=hip_device)
    extra = torch.zeros((n, d), device=hip_device)
    _lib.call("fbn_sparse_fixup_dup", _lib.ptr(dup), n, _lib.ptr(gvec), _lib.ptr(extra), _lib.ptr(slot_row), L + 1,
              d, st)
    torch.cuda.synchronize()
    ids = torch.cat([b["item_id"].view(B, 1), b["item_seq"]], 1).reshape(-1)
    slot = (torch.arange(n, device=hip_device) % (L + 1) > 0).long()
    vec = gvec[torch.arange(n, device=hip_device) // (L + 1), slot]           # entry e's vector
    valid = (ids > 0) & (ids < V)
    ref = torch.zeros((V, d), dtype=torch.float64, device=hip_device)
    ref.index_add_(0, ids[valid], vec[valid].double())
    claimers = (slot_row != -1).nonzero().view(-1)
    rows = (slot_row[claimers] & 0x3FFFFFFF).long()
    flagged = (slot_row[claimers] & 0x40000000) != 0
    got = vec[claimers].double() + torch.where(flagged[:, None], extra[claimers].double(), torch.zeros_like(ref[:1]))
    assert torch.equal(torch.sort(rows).values, torch.unique(ids[valid]))      # each touched row claimed once
    scale = ref[rows].abs().max(1, keepdim=True).values.clamp_min(1.0)
    err = ((got - ref[rows]).abs() / scale).max().item()
    assert err <= 1e-5, err
    if zipf > 0:
        assert int((dup >= 0).sum()) > n // 10       # the case is really duplicate-heavy


@pytest.mark.parametrize("d", [128, 16, 64])
def test_bf16_weight_images_match_torch(hip_device, d):
    """fbn_convert_bf16 (the step's bf16 GEMM operand images, four outputs per thread): every
    image equals torch's round-to-nearest-even bf16 of the same f32 weights, remapped / transposed
    as the GEMMs read them (mlp.0.weight without its V_0 and (0, j) pair columns)."""
    from ctr_recommendation_amd.model_fibinet import build_model
    torch.manual_seed(3)
    p = {k: v.to(hip_device) for k, v in build_model(None, {"embedding_dim": d, "vocab_size": 50}).state_dict().items()}
    x = torch.randn((300, 128), device=hip_device)
    out = ops.bf16_weights(p, d, {}, ops._lib.stream_handle(hip_device), x=x)
    torch.cuda.synchronize()
    w0 = p["mlp.0.weight"]
    cols = torch.cat([torch.arange(d, 6 * d), torch.arange(11 * d, 21 * d)]).to(hip_device)
    ref = {"Wa": w0[:, cols], "WaT": w0[:, cols].T, "Wb": p["mlp.4.weight"], "WbT": p["mlp.4.weight"].T,
           "Wp": p["mm_proj.0.weight"], "W": p["bilinear.W"], "WT": p["bilinear.W"].T, "x": x}
    for k, r in ref.items():
        assert torch.equal(out[k], r.contiguous().bfloat16()), k


@pytest.mark.gpu
def test_gemm_slabs_group_matches_separate_launches(hip_device):
    """fbn_gemm_slabs_group writes exactly the K-slabs separate fbn_gemm_slabs launches write, for
    the step's weight-gradient shapes (C3 at B = 1024 and C2), the split-operand [B | B2] form of
    the MLP input's included."""
    import ctypes
    from ctr_recommendation_amd import _lib
    import os
    st = _lib.stream_handle(hip_device)
    g = torch.Generator(device="cpu").manual_seed(5)
    lib = _lib.lib()
    saved_div = os.environ.get("FBN_GROUP_SPLIT_DIV")
    os.environ["FBN_GROUP_SPLIT_DIV"] = "1"     # the group on fbn_gemm_slabs's K partition
    try:
        _slabs_group_cases(hip_device, st, g, lib, _lib)
    finally:
        if saved_div is None:
            os.environ.pop("FBN_GROUP_SPLIT_DIV", None)
        else:
            os.environ["FBN_GROUP_SPLIT_DIV"] = saved_div


def _slabs_group_cases(hip_device, st, g, lib, _lib):
    import ctypes
    for probs in ([(256, 512, 1024, 0), (512, 1920, 1024, 640), (128, 128, 5120, 0), (128, 128, 1024, 0)],
                  [(256, 512, 512, 0), (512, 240, 512, 0), (16, 16, 2560, 0), (16, 128, 512, 0)]):
        descs, refs, outs = [], [], []
        for (M, N, K, nseg) in probs:
            A = torch.randn(K, M, generator=g).to(hip_device, torch.bfloat16)     # k-major A (transA)
            Bm = torch.randn(K, N, generator=g).to(hip_device, torch.bfloat16)    # k-major B
            B1, B2 = (Bm[:, :nseg].contiguous(), Bm[:, nseg:].contiguous()) if nseg else (Bm, None)
            nbytes = lib.fbn_gemm_slabs_size(M, N, K)
            ns = lib.fbn_gemm_slabs_split(M, N, K)
            ws_ref = torch.full((nbytes // 4,), float("nan"), device=hip_device)
            ws_grp = torch.full((nbytes // 4,), float("nan"), device=hip_device)
            nsp = ctypes.c_int(0)
            ldb = nseg if nseg else N
            _lib.call("fbn_gemm_slabs", _lib.ptr(A), _lib.ptr(B1), M, N, K, M, ldb, 1, 0, _lib.ptr(ws_ref), nbytes, None,
                      0, 0x7FFFFFFF, _lib.ptr(B2) if nseg else None, N - nseg if nseg else 0,
                      nseg if nseg else 0x7FFFFFFF, ctypes.byref(nsp), st)
            assert nsp.value == ns
            descs.append(ops._SlabGemm(A.data_ptr(), B1.data_ptr(), ws_grp.data_ptr(), nbytes, 0,
                                       B2.data_ptr() if nseg else 0, M, N, K, M, ldb, 1, 0, 0, 0,
                                       N - nseg if nseg else 0, nseg if nseg else 0x7FFFFFFF, 0))
            refs.append((ws_ref, ns * M * N))
            outs.append((ws_grp, A, B1, B2))
        arr = (ops._SlabGemm * len(descs))(*descs)
        _lib.call("fbn_gemm_slabs_group", ctypes.addressof(arr), len(descs), st)
        torch.cuda.synchronize()
        for (ref, n), (grp, *_), pr in zip(refs, outs, probs):
            assert torch.equal(ref[:n], grp[:n]), (pr, (ref[:n] - grp[:n]).abs().max().item(),
                                                   torch.isnan(grp[:n]).sum().item())


@pytest.mark.gpu
def test_gemm_slabs_group_default_partition_sums(hip_device):
    """With its default K partition (3/4 of fbn_gemm_slabs's slabs) the group's slab SUM -- what the
    step's sum launch turns into the weight gradient -- equals the separate launch's within fp32
    rounding of a K-long dot product (1e-5 relative to the largest entry)."""
    import ctypes
    import os
    from ctr_recommendation_amd import _lib
    assert "FBN_GROUP_SPLIT_DIV" not in os.environ
    st = _lib.stream_handle(hip_device)
    g = torch.Generator(device="cpu").manual_seed(9)
    lib = _lib.lib()
    for (M, N, K) in ((512, 1920, 8192), (256, 512, 8192), (128, 128, 40960), (128, 128, 8192)):
        A = torch.randn(K, M, generator=g).to(hip_device, torch.bfloat16)
        Bm = torch.randn(K, N, generator=g).to(hip_device, torch.bfloat16)
        nbytes = lib.fbn_gemm_slabs_size(M, N, K)
        ns, ng = lib.fbn_gemm_slabs_split(M, N, K), lib.fbn_gemm_slabs_group_split(M, N, K)
        assert 1 <= ng <= ns
        ws_ref = torch.zeros((nbytes // 4,), device=hip_device)
        ws_grp = torch.zeros((nbytes // 4,), device=hip_device)
        nsp = ctypes.c_int(0)
        _lib.call("fbn_gemm_slabs", _lib.ptr(A), _lib.ptr(Bm), M, N, K, M, N, 1, 0, _lib.ptr(ws_ref), nbytes, None, 0,
                  0x7FFFFFFF, None, 0, 0x7FFFFFFF, ctypes.byref(nsp), st)
        arr = (ops._SlabGemm * 1)(ops._SlabGemm(A.data_ptr(), Bm.data_ptr(), ws_grp.data_ptr(), nbytes, 0, 0, M, N, K,
                                                M, N, 1, 0, 0, 0, 0, 0x7FFFFFFF, 0))
        _lib.call("fbn_gemm_slabs_group", ctypes.addressof(arr), 1, st)
        torch.cuda.synchronize()
        ref = ws_ref[:ns * M * N].view(ns, M, N).sum(0)
        grp = ws_grp[:ng * M * N].view(ng, M, N).sum(0)
        exact = A.float().t() @ Bm.float()
        assert (grp - ref).abs().max().item() <= 1e-5 * exact.abs().max().item(), (M, N, K)


@pytest.mark.gpu
def test_kernel_span_probe(hip_device):
    """fbn_probe_arm / _disarm / _elapsed (bench.py's roofline timings): a probed call's span is its
    kernels' own start-to-end time -- positive, and no longer than host-side events around the same
    call (which add marker packets and dispatch latency); a call that launches nothing leaves the
    probe untaken (-1); an unarmed launch records nothing."""
    from ctr_recommendation_amd import _lib
    M, N, K = 8192, 512, 1920
    A = torch.randn((M, K), device=hip_device).bfloat16()
    W = torch.randn((N, K), device=hip_device).bfloat16()
    C = torch.empty((M, N), device=hip_device)
    ops.gemm(A, W, C, M, N, K, K, K, N, False, True)          # warm-up
    spans, outer = [], []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        kp = _lib.KernelProbe()
        ops.gemm(A, W, C, M, N, K, K, K, N, False, True)
        kp.done()
        e1.record()
        torch.cuda.synchronize()
        assert kp.elapsed_time() > 0
        spans.append(kp.elapsed_time())
        outer.append(e0.elapsed_time(e1))
    assert all(0 < s <= o for s, o in zip(spans, outer)), (spans, outer)
    empty = _lib.KernelProbe()
    ops.gemm(A, W, C, 0, N, K, K, K, N, False, True)          # M = 0: no launch
    empty.done()
    assert empty.elapsed_time() == -1.0
    ops.gemm(A, W, C, M, N, K, K, K, N, False, True)          # unarmed: the last slot stays as it was
    torch.cuda.synchronize()
    assert kp.elapsed_time() == spans[-1]


@pytest.mark.gpu
@pytest.mark.parametrize("M", [8192, 4096])
def test_gemm_bn_bwd_part_epilogue(hip_device, M):
    """fbn_gemm_bn_bwd_part (the BN1 backward's first pass in the epilogue of its dgrad GEMM): C is the
    plain bf16 GEMM, and part[chunk][0 / 1][n] = the chunk's sum of dy / (x - mean) dy with
    dy = (hact > 0) C scale, against torch in float64.  M = 8192 (C3): one 32-row chunk per wave;
    M = 4096 (C2): two 16-row chunks per wave."""
    from ctr_recommendation_amd import _lib
    N, K = 512, 256
    assert _lib.lib().fbn_gemm_bn_bwd_part_supported(M, N, K, K, K, 0, 1)
    g = torch.Generator(device="cpu").manual_seed(9)
    A = torch.randn((M, K), generator=g).to(hip_device).bfloat16()
    W = torch.randn((N, K), generator=g).to(hip_device).bfloat16()
    hact16 = torch.randn((M, N), generator=g).to(hip_device).bfloat16()
    xpre = torch.randn((M, N), generator=g).to(hip_device)
    mean = torch.randn((N,), generator=g).to(hip_device) * 0.1
    nch = _lib.lib().fbn_bn_bwd_chunks(M, N)
    part = torch.full((nch, 3, N), float("nan"), dtype=torch.float64, device=hip_device)
    C = torch.empty((M, N), device=hip_device)
    scale = 1.25
    _lib.call("fbn_gemm_bn_bwd_part", _lib.ptr(A), _lib.ptr(W), _lib.ptr(C), M, N, K, K, K, N, 0, 1,
              _lib.ptr(hact16), _lib.ptr(xpre), _lib.ptr(mean), scale, _lib.ptr(part), _lib.stream_handle(hip_device))
    C0 = torch.empty_like(C)
    ops.gemm(A, W, C0, M, N, K, K, K, N, False, True)
    torch.cuda.synchronize()
    assert torch.equal(C, C0)
    dy = torch.where(hact16.float() > 0, C.double() * scale, torch.zeros_like(C, dtype=torch.float64))
    rpc = M // nch
    s0 = dy.view(nch, rpc, N).sum(1)
    s1 = ((xpre.double() - mean.double()) * dy).view(nch, rpc, N).sum(1)
    assert torch.allclose(part[:, 0], s0, rtol=1e-5, atol=1e-3)
    assert torch.allclose(part[:, 1], s1, rtol=1e-5, atol=1e-3)
    assert bool((part[:, 2] == 0).all())


@pytest.mark.gpu
@pytest.mark.parametrize("B", [8192, 1000, 37])
def test_fused_head_four_rows_per_wave(hip_device, B):
    """fbn_bn_act_head_fwd with the BN2 backward's first pass (bn_act_head_bwd4_kernel, four rows
    per wave): its forward outputs equal the head launch without the backward pass bit for bit,
    and the backward fed its partials equals the backward that computes them itself
    (bn_bwd_partial4, the same rows in the same order) bit for bit.  B = 1000 / 37: ragged chunks."""
    C, p_drop = 256, 0.3
    dev = hip_device
    g = torch.Generator(device="cpu").manual_seed(11)
    X = (torch.randn((B, C), generator=g) * 2 + 0.3).to(dev)
    mean = X.mean(0)
    inv = 1.0 / torch.sqrt(X.var(0, unbiased=False) + 1e-5)
    gamma = (1 + 0.1 * torch.randn((C,), generator=g)).to(dev)
    beta = (0.1 * torch.randn((C,), generator=g)).to(dev)
    hw = (torch.randn((C,), generator=g) / 16).to(dev)
    hb = torch.randn((1,), generator=g).to(dev)
    labels = (torch.rand((B,), generator=g) < 0.4).float().to(dev)
    rng = torch.tensor([0x1234_5678_9abc, 7], dtype=torch.int64).to(dev)
    st = _lib.stream_handle(dev)
    bscale = 1.0 / (1.0 - p_drop)

    def run(with_part):
        out = {k: torch.full((B,), float("nan"), device=dev) for k in ("logits", "probs", "lt", "go")}
        out["Y"] = torch.full((B, C), float("nan"), device=dev)
        out["mask"] = torch.full((B, C), 7, dtype=torch.uint8, device=dev)
        nch = _lib.lib().fbn_bn_bwd_chunks(B, C)
        part = torch.full((nch * 3 * C,), float("nan"), dtype=torch.float64, device=dev) if with_part else None
        _lib.call("fbn_bn_act_head_fwd", _lib.ptr(X), _lib.ptr(out["Y"]), B, C, _lib.ptr(mean), _lib.ptr(inv),
                  _lib.ptr(gamma), _lib.ptr(beta), p_drop, _lib.ptr(rng), 2, _lib.ptr(out["mask"]), None,
                  _lib.ptr(hw), _lib.ptr(hb), _lib.ptr(out["logits"]), _lib.ptr(out["probs"]), _lib.ptr(labels),
                  _lib.ptr(out["lt"]), _lib.ptr(out["go"]), float(B), _lib.ptr(part), float(bscale), st)
        return out, part

    ref, _ = run(False)
    got, part = run(True)
    torch.cuda.synchronize()
    for k in ref:
        assert torch.equal(ref[k], got[k]), k
    assert 0.55 < got["mask"].float().mean().item() < 0.85

    def backward(part_pre):
        d = {"dpre": torch.empty((B, C), device=dev), "dgamma": torch.empty(C, device=dev),
             "dbeta": torch.empty(C, device=dev), "dw": torch.empty(C, device=dev)}
        ops.bn_backward(None, got["go"], hw, got["Y"], bscale, X, mean, inv, gamma, B, C, float(B), d["dpre"],
                        d["dgamma"], d["dbeta"], d["dw"], ops.NO_COLLECTIVE, st, part_pre=part_pre)
        return d

    own, fed = backward(None), backward(part)
    torch.cuda.synchronize()
    for k in own:
        assert torch.equal(own[k], fed[k]), k
    # and against float64 torch
    dy = torch.where(got["Y"] > 0, got["go"][:, None].double() * hw.double() * bscale, torch.zeros((), dtype=torch.float64,
                                                                                                    device=dev))
    assert torch.allclose(fed["dbeta"].double(), dy.sum(0), rtol=1e-5, atol=1e-6)
    assert torch.allclose(fed["dw"].double(), (got["go"][:, None].double() * got["Y"].double()).sum(0), rtol=1e-5,
                          atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("B,C", [(8192, 1024), (1000, 512), (37, 256)])
def test_bn_act_four_rows_per_wave_matches(hip_device, monkeypatch, B, C):
    """The BN + ReLU + dropout forward with four rows per wave (FBN_BN_ACT_R4=1, read per call)
    writes exactly what the one-row form writes: f32 output, bf16 image (and split images) and the
    dropout mask.  B = 1000 / 37: ragged chunks."""
    dev = hip_device
    g = torch.Generator(device="cpu").manual_seed(12)
    X = torch.randn((B, C), generator=g).to(dev)
    mean = X.mean(0)
    inv = 1.0 / torch.sqrt(X.var(0, unbiased=False) + 1e-5)
    gamma = (1 + 0.1 * torch.randn((C,), generator=g)).to(dev)
    beta = (0.1 * torch.randn((C,), generator=g)).to(dev)
    rng = torch.tensor([0x0bad_cafe_1234, 3], dtype=torch.int64).to(dev)
    st = _lib.stream_handle(dev)

    def run(r4):
        monkeypatch.setenv("FBN_BN_ACT_R4", "1" if r4 else "0")
        Y = torch.full((B, C), float("nan"), device=dev)
        Y16 = torch.full((B, C), 7, dtype=torch.int16, device=dev)
        img = torch.full((2, B, C), 7, dtype=torch.int16, device=dev)
        mask = torch.full((B, C), 9, dtype=torch.uint8, device=dev)
        mask2 = torch.full((B, C), 9, dtype=torch.uint8, device=dev)
        _lib.call("fbn_bn_act_fwd", _lib.ptr(X), _lib.ptr(Y), B, C, _lib.ptr(mean), _lib.ptr(inv), _lib.ptr(gamma),
                  _lib.ptr(beta), 0.5, _lib.ptr(rng), 1, _lib.ptr(mask), None, _lib.ptr(Y16), st)
        _lib.call("fbn_bn_act_fwd_img", _lib.ptr(X), None, B, C, _lib.ptr(mean), _lib.ptr(inv), _lib.ptr(gamma),
                  _lib.ptr(beta), 0.5, _lib.ptr(rng), 1, _lib.ptr(mask2), None, _lib.ptr(img), st)
        torch.cuda.synchronize()
        return Y, Y16, img, mask, mask2

    a, b = run(False), run(True)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert torch.equal(a[3], a[4]) and bool((a[3] <= 1).all())


@pytest.mark.gpu
@pytest.mark.parametrize("B,C", [(8192, 512), (1000, 256)])
def test_bn_backward_reduce_columns_per_block(hip_device, monkeypatch, B, C):
    """The BN backward's chunk reduce on 4 / 8 columns per workgroup (FBN_BN_REDUCE_NC, read per
    call) folds every column's 64 chunk streams in the same fixed order as the default 16: the
    whole backward (dX, dgamma, dbeta, head-weight gradient) is bit-identical."""
    dev = hip_device
    g = torch.Generator(device="cpu").manual_seed(13)
    X = torch.randn((B, C), generator=g).to(dev)
    mean = X.mean(0)
    inv = 1.0 / torch.sqrt(X.var(0, unbiased=False) + 1e-5)
    gamma = (1 + 0.1 * torch.randn((C,), generator=g)).to(dev)
    hact = torch.relu(torch.randn((B, C), generator=g)).to(dev)
    gvec = torch.randn((B,), generator=g).to(dev)
    w = torch.randn((C,), generator=g).to(dev)
    st = _lib.stream_handle(dev)
    outs = []
    for nc in ("16", "4", "8"):
        monkeypatch.setenv("FBN_BN_REDUCE_NC", nc)
        d = [torch.full((B, C), float("nan"), device=dev)] + [torch.full((C,), float("nan"), device=dev)
                                                               for _ in range(3)]
        ops.bn_backward(None, gvec, w, hact, 1.25, X, mean, inv, gamma, B, C, float(B), d[0], d[1], d[2], d[3],
                        ops.NO_COLLECTIVE, st, tag=f"nc{nc}")
        torch.cuda.synchronize()
        outs.append(d)
    for other in outs[1:]:
        for a, b in zip(outs[0], other):
            assert torch.equal(a, b)
    dy = torch.where(hact > 0, gvec[:, None].double() * w.double() * 1.25, torch.zeros((), dtype=torch.float64,
                                                                                          device=dev))
    # dy is formed in float (gvec * w, then * scale) and summed in double: float rounding per term
    assert torch.allclose(outs[0][2].double(), dy.sum(0), rtol=1e-4, atol=1e-3)
