"""HIP path vs the CPU oracle (parity gate).  Run on an MI355X: pytest -m gpu.

Tolerances (north_star): probabilities / logits within 1e-4 (fp32 path); gradients within
1e-4 relative to the largest entry of each tensor (fp32 GEMM / atomic summation order only).
"""
import numpy as np
import pytest
import torch

from ctr_recommendation_amd import ops
from ctr_recommendation_amd.data import make_batch
from ctr_recommendation_amd.model_fibinet import build_model
from oracle.fibinet_oracle import build_model as oracle_build

pytestmark = pytest.mark.gpu

V_SMALL = 5000


def _pair(d, seed=0, honour=None):
    cfg = {"embedding_dim": d, "vocab_size": V_SMALL}
    if honour:
        cfg.update(honour)
        cfg["honour_config"] = True
    torch.manual_seed(seed)
    ref = oracle_build(None, cfg, honour_config=bool(honour))
    torch.manual_seed(seed)
    hip = build_model(None, cfg)
    sd_ref = ref.state_dict()
    for k, v in hip.state_dict().items():
        assert torch.equal(v, sd_ref[k]), f"seeded init differs for {k}"
    return ref, hip


def _to(batch, dev):
    return {k: v.to(dev) for k, v in batch.items()}


@pytest.mark.parametrize("d", [16, 128])
def test_forward_eval_parity(hip_device, d):
    ref, hip = _pair(d)
    batch, _ = make_batch(1, 96, V_SMALL)
    ref.eval()
    hip = hip.to(hip_device).eval()
    with torch.no_grad():
        p_ref = ref(batch)
        p_hip = hip(_to(batch, hip_device)).cpu()
    assert p_hip.shape == p_ref.shape
    assert (p_hip - p_ref).abs().max().item() < 1e-4


@pytest.mark.parametrize("d", [16, 128])
def test_forward_train_parity_injected_masks(hip_device, d):
    ref, hip = _pair(d)
    B = 128
    batch, _ = make_batch(2, B, V_SMALL)
    hip = hip.to(hip_device).train()
    p = {k: v for k, v in hip.state_dict(keep_vars=False).items()}
    p = {k: v.contiguous() for k, v in p.items()}
    cfg = ops.FwdConfig(d=d, L=20, training=True, p_drop=0.2)
    rng = torch.tensor([1234, 7], dtype=torch.int64, device=hip_device)
    masks = {"m1": torch.empty((B, 512), dtype=torch.uint8, device=hip_device),
             "m2": torch.empty((B, 256), dtype=torch.uint8, device=hip_device)}
    acts = ops.forward(p, _to(batch, hip_device), cfg, rng, masks_out=masks)
    m1, m2 = masks["m1"].cpu().float(), masks["m2"].cpu().float()
    keep = torch.cat([m1.flatten(), m2.flatten()]).mean().item()
    assert 0.75 < keep < 0.85, keep                       # Bernoulli(0.8) keep-rate
    ref.train()
    logit_ref = ref(batch, masks=(m1, m2), return_logits=True)
    lh = acts["logits"].cpu()
    assert (lh - logit_ref.detach()).abs().max().item() < 1e-4
    assert (acts["probs"].cpu() - torch.sigmoid(logit_ref.detach())).abs().max().item() < 1e-4
    # BN running statistics updated like torch (momentum 0.1, unbiased var)
    for k in ("mlp.1.running_mean", "mlp.1.running_var", "mlp.5.running_mean", "mlp.5.running_var"):
        assert torch.allclose(p[k].cpu(), ref.state_dict()[k], atol=1e-5, rtol=1e-4), k


def _grad_close(g_hip, g_ref, name, rtol=1e-4):
    scale = max(g_ref.abs().max().item(), 1e-6)
    err = (g_hip - g_ref).abs().max().item()
    assert err <= rtol * scale + 1e-7, f"{name}: max err {err:.3e} vs scale {scale:.3e}"


@pytest.mark.parametrize("d,B", [(16, 128), (128, 128), (16, 32), (16, 40), (16, 100), (128, 48)])
def test_backward_parity_no_dropout(hip_device, d, B):
    """B < 64 and B % 64 != 0: one partial GEMM row tile / BN statistics tile (a rank's slice
    under per-GPU BatchNorm can be that small)."""
    ref, hip = _pair(d, honour={"net_dropout": 0.0})
    batch, labels = make_batch(3, B, V_SMALL)
    hip = hip.to(hip_device).train()
    ref.train()
    loss_fn = torch.nn.BCELoss()
    l_ref = loss_fn(ref(batch), labels)
    l_ref.backward()
    y = hip(_to(batch, hip_device))
    l_hip = loss_fn(y, labels.to(hip_device))
    l_hip.backward()
    assert abs(l_hip.item() - l_ref.item()) < 1e-5
    ref_g = {n: p.grad for n, p in ref.named_parameters()}
    for n, p in hip.named_parameters():
        if ref_g[n] is None:
            assert p.grad is None, n
            continue
        if n in ("mlp.0.bias", "mlp.4.bias"):   # exactly cancelled by the following BatchNorm
            assert p.grad.abs().max().item() < 1e-5, n
            continue
        _grad_close(p.grad.cpu(), ref_g[n], n)


def test_padding_and_empty_history(hip_device):
    """All-padding history -> zero field (count clamps to 1); id 0 never receives a gradient."""
    d = 16
    ref, hip = _pair(d, honour={"net_dropout": 0.0})
    B = 32
    batch, labels = make_batch(4, B, V_SMALL)
    batch["item_seq"][:8] = 0          # all padding
    batch["item_seq"][8:16, :] = 7     # repeated id (scatter collisions)
    batch["item_id"][16:20] = 7
    hip = hip.to(hip_device).train()
    ref.train()
    loss_fn = torch.nn.BCELoss()
    loss_fn(ref(batch), labels).backward()
    loss_fn(hip(_to(batch, hip_device)), labels.to(hip_device)).backward()
    g = hip.item_emb.weight.grad.cpu()
    assert g[0].abs().max().item() == 0.0
    _grad_close(g, ref.item_emb.weight.grad, "item_emb.weight")


def test_out_of_range_id_raises(hip_device):
    _, hip = _pair(16)
    batch, _ = make_batch(5, 16, V_SMALL)
    batch["item_id"][3] = V_SMALL + 10
    hip = hip.to(hip_device).eval()
    with pytest.raises(IndexError):
        with torch.no_grad():
            hip(_to(batch, hip_device))


def test_no_history_key(hip_device):
    ref, hip = _pair(16)
    batch, _ = make_batch(6, 64, V_SMALL)
    del batch["item_seq"]
    ref.eval()
    hip = hip.to(hip_device).eval()
    with torch.no_grad():
        assert (hip(_to(batch, hip_device)).cpu() - ref(batch)).abs().max().item() < 1e-4


@pytest.mark.parametrize("d", [16, 128])
def test_hip_matches_committed_golden_vectors(hip_device, d):
    """HIP path vs the committed oracle fixtures (tests/golden/oracle_d*.npz)."""
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", f"oracle_d{d}.npz"))
    batch = {k: torch.from_numpy(z[k]).to(hip_device)
             for k in ("item_id", "item_seq", "likes_level", "views_level", "item_emb_d128")}
    torch.manual_seed(0)
    hip = build_model(None, {"embedding_dim": d, "vocab_size": 1000}).to(hip_device)
    hip.eval()
    with torch.no_grad():
        pe = hip(batch).cpu().numpy()
    assert np.abs(pe - z["probs_eval"]).max() < 1e-4
    # train mode with the fixture's dropout masks injected into the dropout kernel, then backward
    hip.train()
    p = {k: v for k, v in hip.state_dict().items()}
    B = z["item_id"].shape[0]
    cfg = ops.FwdConfig(d=d, L=20, training=True, p_drop=0.2)
    mi = {"m1": torch.from_numpy(z["mask1"]).to(hip_device), "m2": torch.from_numpy(z["mask2"]).to(hip_device)}
    labels = torch.from_numpy(z["labels"]).to(hip_device)
    acts = ops.forward(p, batch, cfg, None, masks_in=mi, labels=labels)
    assert np.abs(acts["logits"].cpu().numpy() - z["logits_train"]).max() < 1e-4
    loss = acts["loss_terms"].sum().item() / B
    assert abs(loss - float(z["loss"])) < 1e-5
    g = {n: torch.zeros_like(v) for n, v in p.items() if v.dtype == torch.float32}
    table_grad = torch.zeros_like(p["item_emb.weight"])
    ops.backward(p, batch, acts, acts["gout"], g, cfg, table_grad=table_grad)
    g["item_emb.weight"] = table_grad           # the scatter-add into the dense table gradient
    for key in [k for k in z.files if k.startswith("grad/")]:
        n = key[5:]
        ref = torch.from_numpy(z[key])
        _grad_close(g[n].cpu(), ref, n)
    assert torch.equal(table_grad[0].cpu(), torch.zeros(d))      # padding_idx=0 row never written
    for key in [k for k in z.files if k.startswith("gradrows/")]:  # first rows of the largest GEMM's wgrad
        n = key[9:]
        ref = torch.from_numpy(z[key])
        _grad_close(g[n][:ref.shape[0]].cpu(), ref, n)


@pytest.mark.parametrize("d,zipf,tau", [(128, 1.05, 2), (16, 1.2, 3), (128, 0.0, 2)])
def test_hot_row_staging_is_bit_identical(hip_device, d, zipf, tau, monkeypatch):
    """The gather's hot-row LDS staging (FBN_GATHER_HOT, the north star's 'LDS staging of hot
    rows' measured as an A/B variant): a staged row read from LDS is the same f32 row, summed in
    the same slot order, so the forward is bit-identical to the plain gather -- under Zipf ids
    (many staged rows), a steeper skew at d = 16, and uniform ids (few or none)."""
    from ctr_recommendation_amd.data import make_device_batches
    V, B = 20000, 2048
    torch.manual_seed(0)
    hip = build_model(None, {"embedding_dim": d, "vocab_size": V}).to(hip_device).eval()
    (batch, _), = make_device_batches(1, B, V, 20, hip_device, seed=9, zipf=zipf)
    with torch.no_grad():
        p0 = hip(batch)
        monkeypatch.setattr(ops, "_GATHER_HOT", tau)
        p1 = hip(batch)
        p2 = hip(batch)          # counts and the list were cleared after the first staged pass
    assert torch.equal(p0, p1) and torch.equal(p0, p2)


@pytest.mark.parametrize("d", [16, 32, 64, 128, 256])
@pytest.mark.parametrize("mode", ["table", "rows_f32", "rows_bf16"])
@pytest.mark.parametrize("hch", ["5", "10"])
def test_gather_compacted_slots_bit_identical(hip_device, d, mode, hch, monkeypatch):
    """The gather with the live history slots compacted first (FBN_FIELDS_CMP=1: ballot + mbcnt, a
    per-sample LDS list, chunks of live rows only) against the plain one on every output of
    fbn_fields_fwd, reading the table (mode 0) or an exchanged row buffer through pos (modes 1 / 2):
    bit-identical (the plain form's padding slots add +0.0); an all-padding sample and a history of
    one live slot included."""
    monkeypatch.setenv("FBN_FIELDS_HCH", hch)
    import ctypes
    from ctr_recommendation_amd._lib import call, ptr
    V, B, L = 5000, 300, 20
    g = torch.Generator().manual_seed(d)
    item = torch.randint(1, V, (B,), generator=g)
    seq = torch.randint(1, V, (B, L), generator=g)
    seq[torch.rand((B, L), generator=g) < 0.5] = 0
    seq[0] = 0                                  # all padding
    seq[1] = 0
    seq[1, 7] = 11                              # one live slot, mid-history
    likes = torch.randint(0, 11, (B,), generator=g)
    views = torch.randint(0, 11, (B,), generator=g)
    dev = hip_device
    f = lambda t: t.to(dev).contiguous()
    item, seq, likes, views = f(item), f(seq), f(likes), f(views)
    hmm = f(torch.randn(B, d, generator=g))
    ln_g, ln_b = f(torch.rand(d, generator=g) + 0.5), f(torch.randn(d, generator=g) * 0.1)
    cate = f(torch.randn(11, d, generator=g))
    table = f(torch.randn(V, d, generator=g))
    w1, b1 = f(torch.randn(3, 6, generator=g)), f(torch.randn(3, generator=g))
    w2, b2 = f(torch.randn(6, 3, generator=g)), f(torch.randn(6, generator=g))
    pos = None
    rows = table
    if mode != "table":
        # every (sample, slot) gets its own row of a shuffled row buffer; padding slots -1
        ids = torch.cat([item[:, None], seq], 1)
        perm = torch.randperm(B * (L + 1), generator=g).to(dev).view(B, L + 1).int()
        pos = torch.where(ids > 0, perm, torch.full_like(perm, -1)).contiguous()
        rows = torch.zeros(B * (L + 1), d, device=dev)
        live = pos >= 0
        rows[pos[live].long()] = table[ids[live]]
        if mode == "rows_bf16":
            rows = rows.bfloat16()

    def run():
        out = {"X": torch.full((B, 2, d), 7.0, device=dev), "Vc": torch.full((B, 5, d), 7.0, device=dev),
               "a": torch.zeros(B, 6, device=dev), "cnt": torch.zeros(B, device=dev)}
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        call("fbn_fields_fwd", ptr(item), ptr(seq), ptr(likes), ptr(views), ptr(hmm), ptr(ln_g), ptr(ln_b), 1e-5,
             ptr(cate), 11, ptr(rows), V if mode == "table" else B * (L + 1), ptr(pos), ptr(w1), ptr(b1), ptr(w2),
             ptr(b2), 3, ptr(out["X"]), ptr(out["Vc"]), None, None, 0, 0, ptr(out["a"]), ptr(out["cnt"]), ptr(err),
             None, None, B, L, d, int(mode == "rows_bf16"), torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize()
        assert int(err.item()) == 0
        return out
    old = run()
    monkeypatch.setenv("FBN_FIELDS_CMP", "1")
    new = run()
    for k in ("X", "Vc", "a", "cnt"):
        assert torch.equal(new[k], old[k]), k
    assert new["cnt"][0].item() == 1.0 and new["cnt"][1].item() == 1.0
    # all padding: the history mean is exactly zero; one live slot: exactly that row
    assert torch.all(new["X"][0, 1] == 0)
    ref1 = (rows[pos[1, 8].long()].float() if mode != "table" else table[11])
    assert torch.equal(new["X"][1, 1], ref1)
