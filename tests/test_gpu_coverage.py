"""Parity tests that reach the branches the per-kernel tests do not (pytest -m gpu, MI355X).

* the clip coefficient engaged (max_norm lowered so coef < 1) in the native trainer -- immediate
  and deferred table gradients -- and in the drop-in under the reference loop verbatim
  (torch Adam + clip_grad_norm_ + OneCycleLR, src/train_fibinet.py:78-92,113-123);
* AUC of the HIP path vs the oracle on the same 65 536-sample eval set after training steps
  (north star: |dAUC| <= 1e-4 for fp32 and bf16_fwd; the all-bf16 dAUC is recorded and held to
  its measured value plus margin);
* the BCE log clamp (p rounding to exactly 0 or 1, src/train_fibinet.py:79 BCELoss);
* the configs' full shapes: C2 (d=16, V=1M, B=4096) and C3 (d=128, V=1.25M, B=8192) through
  the drop-in forward + backward and one native-trainer step, against the oracle;
* the opt-in config surface on the GPU: bilinear_type "each", senet_reduction 3
  (src/model_fibinet.py:13,52-56,81-86);
* nn.DataParallel's replica (src/train_fibinet.py:69-70): forward + backward through a
  torch.nn.parallel.replicate() copy;
* the device-side step bound (graph replays past total_steps).

Tolerances are written next to each assert.
"""
import numpy as np
import pytest
import torch

from ctr_recommendation_amd.data import make_batch
from ctr_recommendation_amd.model_fibinet import build_model
from ctr_recommendation_amd.trainer import FiBiNETTrainer
from ctr_recommendation_amd.utils import compute_auc
from oracle.fibinet_oracle import OracleTrainer, build_model as oracle_build, compute_auc as oracle_auc

pytestmark = pytest.mark.gpu
NO_DROP = {"honour_config": True, "net_dropout": 0.0}


def _to(b, dev):
    return {k: v.to(dev) for k, v in b.items()}


def _grad_close(g_hip, g_ref, name, rtol=1e-4):
    scale = max(g_ref.abs().max().item(), 1e-6)
    err = (g_hip - g_ref).abs().max().item()
    assert err <= rtol * scale + 1e-7, f"{name}: max err {err:.3e} vs scale {scale:.3e}"


def _trainers(d, V, B, hip_device, total=50, max_norm=10.0, **kw):
    cfg = dict({"embedding_dim": d, "vocab_size": V}, **NO_DROP)
    torch.manual_seed(0)
    ref = oracle_build(None, cfg, honour_config=True)
    init = {k: v.clone() for k, v in ref.state_dict().items()}
    otr = OracleTrainer(ref, lr=1e-3, weight_decay=1e-5, total_steps=total, max_norm=max_norm)
    htr = FiBiNETTrainer(cfg, total_steps=total, batch_size=B, device=hip_device, max_norm=max_norm,
                         init_state={k: v.clone() for k, v in init.items()}, **kw)
    return ref, otr, htr


# ---------------------------------------------------------------- clip engaged
@pytest.mark.parametrize("defer", [True, False])
@pytest.mark.parametrize("d", [16, 128])
def test_clip_engaged_trainer_matches_reference_loop(hip_device, d, defer):
    """max_norm 0.05 (gradient norms here are ~1): every step runs with clip coef < 1, and the
    deferred table gradients replay with the coefficient of the step that produced them
    (coef_hist).  Rows recur (V = 3000) and the window is small (4) so deferred vectors are
    consumed by claims and by windows.  Gates as test_gpu_trainer: loss 2e-5 at step 0, 5e-4
    after; eval probabilities of the updated models 2e-3."""
    V, B = 3000, 256
    ref, otr, htr = _trainers(d, V, B, hip_device, max_norm=0.05, lazy_window=4, defer_table_grads=defer)
    assert htr.deferred == defer
    for s in range(6):
        b, y = make_batch(500 + s, B, V)
        lh = htr.step(_to(b, hip_device), y.to(hip_device)).item()
        lr_, _ = otr.step(b, y)
        assert otr.last_total_norm > 0.05 * 4, "clip must engage"
        coef = htr.coef.item()
        assert coef < 0.5, coef
        # the coefficient from the HIP norm vs the oracle's: 1e-4 relative on the shared init,
        # 2e-2 once the two trajectories carry Adam's noise-level sign flips
        tol = 1e-4 if s == 0 else 2e-2
        assert abs(coef - min(1.0, 0.05 / (otr.last_total_norm + 1e-6))) < tol * coef + 1e-7, \
            (s, coef, otr.last_total_norm)
        assert abs(lh - lr_) < (2e-5 if s == 0 else 5e-4), (s, lh, lr_)
    htr.check_ids()
    b, _ = make_batch(999, 512, V)
    ref.eval()
    with torch.no_grad():
        pr = ref(b)
    ph = htr.predict(_to(b, hip_device)).cpu()
    assert (pr - ph).abs().max().item() < 2e-3


@pytest.mark.parametrize("max_norm", [10.0, 0.01])
def test_deferred_vs_immediate_bit_identical_with_clip(hip_device, max_norm):
    """Deferred table gradients replayed at a row's next visit == applied at the end of their
    step, bit for bit, also when every step's gradient is scaled by a clip coefficient < 1
    (no duplicate ids within a step, so no float-atomic folds)."""
    V, B, L, steps = 40000, 64, 20, 12
    cfg = {"embedding_dim": 128, "vocab_size": V}
    torch.manual_seed(0)
    init = oracle_build(None, cfg).state_dict()
    kw = dict(total_steps=20, batch_size=B, device=hip_device, init_state=init, lazy_window=4, max_norm=max_norm)
    imm = FiBiNETTrainer(cfg, defer_table_grads=False, **kw)
    dfr = FiBiNETTrainer(cfg, defer_table_grads=True, **kw)
    g = torch.Generator().manual_seed(7)
    pool = torch.randperm(V - 1, generator=g)[:3000] + 1
    coefs = []
    for s in range(steps):
        b, y = make_batch(300 + s, B, V)
        ids = pool[torch.randperm(len(pool), generator=g)[:B * (L + 1)]].view(B, L + 1)
        b["item_id"] = ids[:, 0].clone()
        seq = ids[:, 1:].clone()
        seq[b["item_seq"] == 0] = 0
        b["item_seq"] = seq
        db = _to(b, hip_device)
        l1, l2 = imm.step(db, y.to(hip_device)).item(), dfr.step(db, y.to(hip_device)).item()
        assert l1 == l2, (s, l1, l2)
        coefs.append(dfr.coef.item())
    if max_norm < 1:
        assert max(coefs) < 1.0, coefs
    imm.flush()
    dfr.flush()
    torch.cuda.synchronize()
    for a, c in ((imm.E, dfr.E), (imm.Em, dfr.Em), (imm.Ev, dfr.Ev), (imm.flat_p, dfr.flat_p)):
        assert torch.equal(a, c)


@pytest.mark.parametrize("max_norm", [10.0, 0.05])
def test_dropin_under_reference_loop_verbatim(hip_device, max_norm):
    """The reference's loop body (train_fibinet.py:113-123) run verbatim -- torch.optim.Adam(L2),
    BCELoss, clip_grad_norm_, OneCycleLR -- over the drop-in module on the GPU and over the
    oracle on the CPU, 5 steps.  Bars: loss 2e-5 at step 0 and 5e-4 after; the clip norms
    agree to 1e-4 relative at step 0 and 2e-2 after; eval probabilities 2e-3 after the loop."""
    d, V, B, total = 16, 3000, 256, 40
    cfg = dict({"embedding_dim": d, "vocab_size": V}, **NO_DROP)
    models = []
    for dev in ("cpu", hip_device):
        torch.manual_seed(0)
        m = (oracle_build(None, cfg, honour_config=True) if dev == "cpu" else build_model(None, cfg)).to(dev)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
        sch = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=1e-2, total_steps=total, pct_start=0.3,
                                                  div_factor=25.0, final_div_factor=1000.0)
        models.append((m, opt, sch, dev))
    loss_fn = torch.nn.BCELoss()
    for s in range(5):
        b, y = make_batch(40 + s, B, V)
        out = []
        for m, opt, sch, dev in models:
            m.train()
            opt.zero_grad()
            loss = loss_fn(m(_to(b, dev)), y.to(dev))
            loss.backward()
            norm = torch.nn.utils.clip_grad_norm_(m.parameters(), max_norm=max_norm)
            opt.step()
            sch.step()
            out.append((loss.item(), float(norm)))
        (lr_, nr), (lh, nh) = out
        assert abs(lh - lr_) < (2e-5 if s == 0 else 5e-4), (s, lh, lr_)
        assert abs(nh - nr) <= (1e-4 if s == 0 else 2e-2) * nr, (s, nh, nr)
        if max_norm < 1:
            assert nr > 4 * max_norm
    b, _ = make_batch(77, 512, V)
    (mr, *_), (mh, *_) = models
    mr.eval()
    mh.eval()
    with torch.no_grad():
        assert (mr(b) - mh(_to(b, hip_device)).cpu()).abs().max().item() < 2e-3


# ---------------------------------------------------------------- AUC parity
def _eval_auc(predict, V, n=65536, chunk=8192, seed=4242):
    ys, ps = [], []
    for i in range(n // chunk):
        b, y = make_batch(seed + i, chunk, V, signal="fields")
        ys.append(y.numpy())
        ps.append(predict(b))
    y, p = np.concatenate(ys), np.concatenate(ps)
    return y, p


@pytest.mark.parametrize("d", [16, 128])
def test_auc_parity_after_training(hip_device, d):
    """North star: AUC within 1e-4 of the CPU path on the same synthetic eval set.  4 training
    steps (B = 1024, OneCycle over 40 steps) from the same init on a learnable planted signal
    (AUC 0.85-0.87), then eval-mode probabilities on 65 536 samples.  Checked twice: (a) the two
    independently trained models (trajectory parity); (b) the HIP-trained weights loaded into
    the oracle (forward parity of the evaluation itself).  Why 4 steps: Adam's sign-like early
    updates make any two fp32 trajectories drift -- the fp32 CPU oracle itself is 2.5e-6 AUC from
    a float64 oracle after 4 steps at d=128, 8.4e-5 after 8 and 7.2e-5 after 24 at d=16
    (measured on this eval set) -- so a 1e-4 trajectory bar is meaningful only while that drift
    is well inside it."""
    V, B = 20000, 1024
    ref, otr, htr = _trainers(d, V, B, hip_device, total=40)
    for s in range(4):
        b, y = make_batch(800 + s, B, V, signal="fields")
        htr.step(_to(b, hip_device), y.to(hip_device))
        otr.step(b, y)
    ref.eval()

    def pr(m):
        def f(b):
            with torch.no_grad():
                return m(b).numpy()
        return f
    y, p_ref = _eval_auc(pr(ref), V)
    _, p_hip = _eval_auc(lambda b: htr.predict(_to(b, hip_device)).cpu().numpy(), V)
    a_ref, a_hip = oracle_auc(y, p_ref), compute_auc(y, p_hip)
    print(f"d={d}: AUC oracle {a_ref:.6f} HIP {a_hip:.6f} dAUC {abs(a_hip - a_ref):.2e} "
          f"max|dp| {np.abs(p_hip - p_ref).max():.2e}")
    assert a_ref > 0.55, a_ref                           # the models learned the planted signal
    assert abs(a_hip - a_ref) <= 1e-4, (a_hip, a_ref)
    # (b) the same (HIP-trained) weights through the oracle's forward
    twin = oracle_build(None, dict({"embedding_dim": d, "vocab_size": V}, **NO_DROP), honour_config=True)
    twin.load_state_dict(htr.state_dict())
    twin.eval()
    _, p_twin = _eval_auc(pr(twin), V)
    assert np.abs(p_hip - p_twin).max() < 1e-4
    assert abs(compute_auc(y, p_hip) - oracle_auc(y, p_twin)) <= 1e-5


# bars of the compute modes (profiles/r03_auc_parity*.json hold the measured values)
PRECISION_MODES = ("fp32", "bf16_fwd", "bf16")
EVAL_AUC_BAR = 1e-4           # the same weights evaluated by the mode vs by the fp32 oracle
TRAJ_AUC_BAR = {"fp32": 1e-4, "bf16_fwd": 1e-4, "bf16": 1e-4}   # 4 training steps, vs the fp32 oracle


@pytest.mark.parametrize("shape", ["small", "C3"])
def test_auc_precision_modes_vs_oracle(hip_device, shape):
    """The three compute modes against the oracle (north star: AUC within 1e-4 of the CPU path on
    the same synthetic batch), each trainer driven by the bench's own call: step(b, y,
    next_batch=...) with eager launches.
      fp32      -- the reference's precision;
      bf16_fwd  -- C3's "bf16 fwd / fp32 grad accum": forward GEMM operands bf16, backward fp32;
      bf16      -- the benched headline mode: every GEMM operand bf16 (forward and backward).
    small: d 128, V 20 000, B 1024; C3: d 128, V 1.25 M, B 8192 (the config's own shape).
    Measured, on the 65 536-sample eval set:
      (a) evaluation parity: each mode's trained weights evaluated by the mode's own forward vs the
          SAME weights through the fp32 oracle forward -- |dAUC| <= 1e-4 (pure forward precision);
      (b) trajectory parity after 4 steps from one init: the mode's model vs the fp32 oracle's --
          |dAUC| <= 1e-4;
      (c) reported, not gated: the same after 8 steps, with the fp32 CPU oracle's own distance to a
          float64 oracle beside it.  Adam's first updates are sign(g) * lr per element, so any two
          trajectories -- fp32 CPU vs float64 included -- drift apart at a rate set by gradients
          at rounding level, not by the mode's precision.
    Everything is written to $FBN_PARITY_OUT/auc_parity_<shape>.json (default gpurun_out/parity/)."""
    import json
    import os
    d = 128
    V, B = (20000, 1024) if shape == "small" else (1_250_000, 8192)
    cfg = dict({"embedding_dim": d, "vocab_size": V}, **NO_DROP)
    torch.manual_seed(0)
    ref = oracle_build(None, cfg, honour_config=True)
    init = {k: v.clone() for k, v in ref.state_dict().items()}
    r64 = oracle_build(None, cfg, honour_config=True).double()
    r64.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in init.items()})
    otr, o64 = OracleTrainer(ref, total_steps=40), OracleTrainer(r64, total_steps=40)
    htrs = {m: FiBiNETTrainer(dict(cfg, compute_dtype=m), total_steps=40, batch_size=B, device=hip_device,
                              init_state=init) for m in PRECISION_MODES}
    del init

    def pr(m, dbl=False):
        def f(b):
            with torch.no_grad():
                bb = {k: (v.double() if (dbl and v.is_floating_point()) else v) for k, v in b.items()}
                return m(bb).float().numpy()
        return f
    rec = {"shape": {"d": d, "V": V, "B": B, "eval_samples": 65536}, "eval_bar": EVAL_AUC_BAR,
           "call": "FiBiNETTrainer.step(b, y, next_batch=<following batch>), eager launches (bench.py's timed "
                   "call: next-batch prefetch + pre-claims, side-stream window / prefetch, duplicate fold on the "
                   "side stream)",
           "trajectory_bar": TRAJ_AUC_BAR, "steps": {}}
    # the bench's own call (bench.py run_step, eager): step(b, y, next_batch=<the following batch>), so
    # the next-batch table-Adam prefetch with its tagged pre-claims, the side-stream passes and the
    # duplicate-gradient fold on the side stream all run inside the parity check
    host = [make_batch(800 + s, B, V, signal="fields") for s in range(9)]
    dev_b = [(_to(b, hip_device), y.to(hip_device)) for b, y in host]
    for s in range(8):
        b, y = host[s]
        db, dy = dev_b[s]
        for htr in htrs.values():
            htr.step(db, dy, next_batch=dev_b[s + 1][0])
        otr.step(b, y)
        o64.step({k: v.double() if v.is_floating_point() else v for k, v in b.items()}, y.double())
        print(f"[{shape}] step {s} done", flush=True)
        if s + 1 not in (4, 8):
            continue
        ref.eval()
        r64.eval()
        yv, p_ref = _eval_auc(pr(ref), V)
        _, p64 = _eval_auc(pr(r64, True), V)
        a_ref = oracle_auc(yv, p_ref)
        st = {"oracle_auc": a_ref, "fp32_oracle_vs_f64_dAUC": abs(a_ref - oracle_auc(yv, p64)), "modes": {}}
        for mode, htr in htrs.items():
            _, p_hip = _eval_auc(lambda bt: htr.predict(_to(bt, hip_device)).cpu().numpy(), V)
            twin = oracle_build(None, cfg, honour_config=True)
            twin.load_state_dict(htr.state_dict())
            twin.eval()
            _, p_twin = _eval_auc(pr(twin), V)
            a_hip = compute_auc(yv, p_hip)
            st["modes"][mode] = {"auc": a_hip, "trajectory_dAUC": abs(a_hip - a_ref),
                                 "trajectory_max_abs_dp": float(np.abs(p_hip - p_ref).max()),
                                 "eval_dAUC": abs(a_hip - oracle_auc(yv, p_twin)),
                                 "eval_max_abs_dp": float(np.abs(p_hip - p_twin).max()),
                                 "eval_mean_abs_dp": float(np.abs(p_hip - p_twin).mean())}
            del twin
        rec["steps"][s + 1] = st
        print(json.dumps({s + 1: st}), flush=True)
        ref.train()
        r64.train()
    out = os.environ.get("FBN_PARITY_OUT", os.path.join("gpurun_out", "parity"))
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, f"auc_parity_{shape}.json"), "w") as f:
        json.dump(rec, f, indent=1)
    assert rec["steps"][4]["oracle_auc"] > 0.55
    for mode in PRECISION_MODES:
        for n in (4, 8):
            r = rec["steps"][n]["modes"][mode]
            assert r["eval_dAUC"] <= EVAL_AUC_BAR, (n, mode, r)
        r = rec["steps"][4]["modes"][mode]
        assert r["trajectory_dAUC"] <= TRAJ_AUC_BAR[mode], (mode, r)


# ---------------------------------------------------------------- BCE clamp
@pytest.mark.parametrize("bias", [120.0, -120.0, 16.0])
def test_bce_saturation(hip_device, bias):
    """Head bias forced so p = sigmoid(o) rounds to exactly 1 (bias 120) or 0 (-120): BCELoss
    clamps the log at -100 and the gradient through sigmoid is exactly 0 (ATen:
    (p-t)/max(p(1-p),1e-12) * p(1-p)).  bias 16: p = 1 - 1.1e-7, just unsaturated."""
    d, V, B = 16, 3000, 256
    cfg = dict({"embedding_dim": d, "vocab_size": V}, **NO_DROP)
    torch.manual_seed(0)
    ref = oracle_build(None, cfg, honour_config=True)
    with torch.no_grad():
        ref.mlp[8].bias.fill_(bias)
    init = {k: v.clone() for k, v in ref.state_dict().items()}
    otr = OracleTrainer(ref, total_steps=10)
    htr = FiBiNETTrainer(cfg, total_steps=10, batch_size=B, device=hip_device, init_state=init)
    for s in range(2):
        b, y = make_batch(60 + s, B, V)
        lh = htr.step(_to(b, hip_device), y.to(hip_device)).item()
        lr_, p = otr.step(b, y)
        if abs(bias) > 100:
            assert bool(((p == 0) | (p == 1)).all())
        assert abs(lh - lr_) <= 1e-5 * max(1.0, lr_), (s, lh, lr_)
    # the drop-in under torch's BCELoss: the clamp and the zero sigmoid gradient
    torch.manual_seed(0)
    hip = build_model(None, cfg).to(hip_device).train()
    with torch.no_grad():
        hip.mlp[8].bias.fill_(bias)
    torch.manual_seed(0)
    ref2 = oracle_build(None, cfg, honour_config=True).train()
    with torch.no_grad():
        ref2.mlp[8].bias.fill_(bias)
    b, y = make_batch(61, B, V)
    loss_fn = torch.nn.BCELoss()
    lr2 = loss_fn(ref2(b), y)
    lr2.backward()
    lh2 = loss_fn(hip(_to(b, hip_device)), y.to(hip_device))
    lh2.backward()
    assert abs(lh2.item() - lr2.item()) <= 1e-5 * max(1.0, lr2.item())
    _grad_close(hip.mlp[8].weight.grad.cpu(), ref2.mlp[8].weight.grad, "mlp.8.weight")


# ---------------------------------------------------------------- config-size shapes
def _untie_relus(cfg, b, tol=1e-5):
    """Bias nudges that keep every pre-ReLU value of batch b at least tol from 0 (float64 oracle).

    At the config shapes a batch holds ~10^6-10^7 pre-ReLU values (mm_proj LayerNorm, SENET
    hidden, BN1, BN2); a few lie within fp32 rounding of 0, where two correct fp32
    implementations take opposite sides of the ReLU -- measured: C2's batch has one BN1 output
    at -4.6e-7, and the fp32 CPU oracle on one host, the HIP path, and f64 disagree on it, which
    moves one sample's gradients by ~4 % (the table rows it touches: 2.3e-2 x max).  The test
    moves such a channel's bias (the ReLU's input offset) to a value where no sample ties, in
    forward order, and gives every model the same nudged weights."""
    torch.manual_seed(0)
    m = oracle_build(None, cfg, honour_config=True).double().train()
    bb = dict(b, item_emb_d128=b["item_emb_d128"].double())
    nudges = {}
    layers = [("mm_proj.1.bias", lambda x, v, c, h1: m.mm_proj[1](m.mm_proj[0](bb["item_emb_d128"]))),
              ("senet.excitation.0.bias", lambda x, v, c, h1: m.senet.excitation[0](x.mean(-1))),
              ("mlp.1.bias", lambda x, v, c, h1: m.mlp[1](m.mlp[0](c))),
              ("mlp.5.bias", lambda x, v, c, h1: m.mlp[5](m.mlp[4](h1)))]
    sd = m.state_dict()
    for name, pre_fn in layers:
        for _ in range(8):
            with torch.no_grad():
                x = m.fields(bb)
                v = m.senet(x)
                c = torch.cat([v.reshape(v.shape[0], -1), m.bilinear(v).reshape(v.shape[0], -1)], 1)
                h1 = torch.relu(m.mlp[1](m.mlp[0](c)))
                pre = pre_fn(x, v, c, h1)
            close = (pre.abs() < tol).any(0).nonzero().flatten().tolist()
            if not close:
                break
            for ch in close:
                col = pre[:, ch]
                for delta in (2e-4, -2e-4, 5e-4, -5e-4, 1e-3, -1e-3, 3e-3, -3e-3):
                    if bool(((col + delta).abs() >= tol).all()):
                        break
                with torch.no_grad():
                    sd[name][ch] += delta
                nudges.setdefault(name, {})[ch] = nudges.get(name, {}).get(ch, 0.0) + delta
    return nudges


def _apply_nudges(model, nudges):
    sd = model.state_dict()
    with torch.no_grad():
        for name, chans in nudges.items():
            for ch, delta in chans.items():
                sd[name][ch] += delta


@pytest.mark.parametrize("cfgname,d,V,B", [("C2", 16, 1_000_000, 4096), ("C3", 128, 1_250_000, 8192)])
def test_config_size_dropin_fwd_bwd(hip_device, cfgname, d, V, B):
    """Full config shapes (grid caps, split-K plans, fields-backward grid all change with B):
    fp32 eval probabilities 1e-4 and loss 1e-5 vs the fp32 oracle; every gradient, the dense
    table gradient (scatter-add, padding row untouched) included, within 1e-4 x its max of a
    FLOAT64 copy of the oracle (the fp32 CPU path's own deviation is printed beside it).  The
    batch is made ReLU-tie-free first (_untie_relus)."""
    cfg = dict({"embedding_dim": d, "vocab_size": V}, **NO_DROP)
    b, y = make_batch(11, B, V)
    nudges = _untie_relus(cfg, b)
    print(f"{cfgname}: ReLU-tie bias nudges {nudges}")
    models = {}
    for kind in ("f32", "f64", "hip"):
        torch.manual_seed(0)
        m = build_model(None, cfg) if kind == "hip" else oracle_build(None, cfg, honour_config=True)
        _apply_nudges(m, nudges)
        models[kind] = m.double() if kind == "f64" else (m.to(hip_device) if kind == "hip" else m)
    db = _to(b, hip_device)
    ref, hip, r64 = models["f32"], models["hip"], models["f64"]
    ref.eval()
    hip.eval()
    with torch.no_grad():
        assert (hip(db).cpu() - ref(b)).abs().max().item() < 1e-4, cfgname
    loss_fn = torch.nn.BCELoss()
    for m in models.values():
        m.train()
    lr_ = loss_fn(ref(b), y)
    lr_.backward()
    lh = loss_fn(hip(db), y.to(hip_device))
    lh.backward()
    assert abs(lh.item() - lr_.item()) < 1e-5
    loss_fn(r64(dict(b, item_emb_d128=b["item_emb_d128"].double())), y.double()).backward()
    ref_g = dict(r64.named_parameters())
    f32_g = dict(ref.named_parameters())
    for n, p in hip.named_parameters():
        if ref_g[n].grad is None:
            assert p.grad is None, n
            continue
        if n in ("mlp.0.bias", "mlp.4.bias"):      # cancelled exactly by the next BatchNorm
            continue
        g64 = ref_g[n].grad
        dev_hip = ((p.grad.cpu().double() - g64).abs().max() / g64.abs().max()).item()
        dev_cpu = ((f32_g[n].grad.double() - g64).abs().max() / g64.abs().max()).item()
        print(f"{cfgname} {n}: HIP {dev_hip:.2e}  fp32 CPU {dev_cpu:.2e} (x max, vs f64)")
        _grad_close(p.grad.cpu().double(), g64, f"{cfgname} {n}")
    assert hip.item_emb.weight.grad[0].abs().max().item() == 0.0


@pytest.mark.parametrize("cfgname,d,V,B,dtype", [("C2", 16, 1_000_000, 4096, "fp32"),
                                                 ("C2", 16, 1_000_000, 4096, "bf16"),
                                                 ("C3", 128, 1_250_000, 8192, "fp32"),
                                                 ("C3", 128, 1_250_000, 8192, "bf16_fwd"),
                                                 ("C3", 128, 1_250_000, 8192, "bf16")])
def test_config_size_trainer_step(hip_device, cfgname, d, V, B, dtype):
    """One native-trainer step + eval forward at the config's shape vs one oracle step.  fp32:
    loss 2e-5, eval probabilities after the step 2e-3 (Adam's first step is sign(g)*lr per
    element), AUC of those probabilities 1e-4.  bf16_fwd / bf16: loss 1e-4 / 2e-3 relative, AUC
    5e-4 -- after one step on an unlearned signal the 8 192-sample eval set is nearly tied, so the
    AUC moves with Adam's sign(g) first update; test_auc_precision_modes_vs_oracle holds the modes to
    1e-4 on 65 536 samples (the values are printed and written to $FBN_PARITY_OUT)."""
    import json
    import os
    cfg = dict({"embedding_dim": d, "vocab_size": V}, **NO_DROP)
    torch.manual_seed(0)
    ref = oracle_build(None, cfg, honour_config=True)
    init = {k: v.clone() for k, v in ref.state_dict().items()}
    otr = OracleTrainer(ref, total_steps=100)
    hcfg = dict(cfg, compute_dtype=dtype)
    htr = FiBiNETTrainer(hcfg, total_steps=100, batch_size=B, device=hip_device, init_state=init)
    del init
    b, y = make_batch(21, B, V)
    lh = htr.step(_to(b, hip_device), y.to(hip_device)).item()
    lr_, _ = otr.step(b, y)
    be, ye = make_batch(22, B, V)
    ref.eval()
    with torch.no_grad():
        pr = ref(be).numpy()
    ph = htr.predict(_to(be, hip_device)).cpu().numpy()
    da = abs(compute_auc(ye.numpy(), ph) - oracle_auc(ye.numpy(), pr))
    rec = {"config": cfgname, "dtype": dtype, "loss_hip": lh, "loss_oracle": lr_, "rel_dloss": abs(lh - lr_) / lr_,
           "dAUC": da, "max_abs_dp": float(np.abs(ph - pr).max())}
    print(json.dumps(rec))
    out = os.environ.get("FBN_PARITY_OUT", os.path.join("gpurun_out", "parity"))
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, f"one_step_{cfgname}_{dtype}.json"), "w") as f:
        json.dump(rec, f, indent=1)
    if dtype == "fp32":
        assert abs(lh - lr_) < 2e-5, (lh, lr_)
        assert np.abs(ph - pr).max() < 2e-3
        assert da <= 1e-4, da
    elif dtype == "bf16_fwd":
        assert abs(lh - lr_) <= 1e-4 * lr_, (lh, lr_)     # measured 3.8e-6
        assert da <= 5e-4, da                             # measured 1.05e-4 (8 192 samples; see below)
    else:
        assert abs(lh - lr_) <= 2e-3 * lr_, (lh, lr_)
        assert da <= 5e-4, da


# ---------------------------------------------------------------- opt-in config surface
@pytest.mark.parametrize("honour", [{"bilinear_type": "each"}, {"senet_reduction": 3},
                                    {"bilinear_type": "each", "senet_reduction": 3}])
@pytest.mark.parametrize("d", [16, 128])
def test_optin_config_surface_parity(hip_device, d, honour):
    """bilinear_type "each" (W_i on field i, model_fibinet.py:81-86) and senet_reduction 3
    (6 -> 2 -> 6, :13), which the reference's config names but its code ignores: fp32 eval
    probabilities 1e-4, gradients 1e-4 x max."""
    V = 5000
    cfg = dict({"embedding_dim": d, "vocab_size": V}, **NO_DROP, **honour)
    torch.manual_seed(0)
    ref = oracle_build(None, cfg, honour_config=True)
    torch.manual_seed(0)
    hip = build_model(None, cfg).to(hip_device)
    sd = ref.state_dict()
    for k, v in hip.state_dict().items():
        assert torch.equal(v.cpu(), sd[k]), k
    b, y = make_batch(8, 128, V)
    ref.eval()
    hip.eval()
    with torch.no_grad():
        assert (hip(_to(b, hip_device)).cpu() - ref(b)).abs().max().item() < 1e-4
    ref.train()
    hip.train()
    loss_fn = torch.nn.BCELoss()
    loss_fn(ref(b), y).backward()
    loss_fn(hip(_to(b, hip_device)), y.to(hip_device)).backward()
    rg = dict(ref.named_parameters())
    for n, p in hip.named_parameters():
        if rg[n].grad is None or n in ("mlp.0.bias", "mlp.4.bias"):
            continue
        _grad_close(p.grad.cpu(), rg[n].grad, n)


# ---------------------------------------------------------------- DataParallel
def test_dataparallel_replica_forward_backward(hip_device):
    """train_fibinet.py:69-70 wraps the model in nn.DataParallel when more than one GPU is
    visible.  A replica made by torch.nn.parallel.replicate (what DataParallel.forward does)
    holds its parameters as plain attributes: forward + backward through it must match the
    oracle and land the gradients on the ORIGINAL parameters."""
    d, V, B = 16, 5000, 128
    cfg = dict({"embedding_dim": d, "vocab_size": V}, **NO_DROP)
    torch.manual_seed(0)
    ref = oracle_build(None, cfg, honour_config=True)
    torch.manual_seed(0)
    hip = build_model(None, cfg).to(hip_device).train()
    replica = torch.nn.parallel.replicate(hip, [hip_device.index or 0])[0]
    assert len(list(replica.parameters())) == 0          # what broke round 1's drop-in
    b, y = make_batch(9, B, V)
    loss_fn = torch.nn.BCELoss()
    ref.train()
    lr_ = loss_fn(ref(b), y)
    lr_.backward()
    lh = loss_fn(replica(_to(b, hip_device)), y.to(hip_device))
    lh.backward()
    assert abs(lh.item() - lr_.item()) < 1e-5
    rg = dict(ref.named_parameters())
    for n, p in hip.named_parameters():
        if rg[n].grad is None or n in ("mlp.0.bias", "mlp.4.bias"):
            continue
        assert p.grad is not None, n
        _grad_close(p.grad.cpu(), rg[n].grad, n)
    # the DataParallel wrapper itself (one device: it calls the module directly)
    dp = torch.nn.DataParallel(hip, device_ids=[hip_device.index or 0])
    hip.eval()
    ref.eval()
    with torch.no_grad():
        assert (dp(_to(b, hip_device)).cpu() - ref(b)).abs().max().item() < 1e-4


def test_dropout_streams_per_device_and_step(hip_device):
    """Dropout draws a fresh mask every forward, also through replicas rebuilt per step."""
    cfg = {"embedding_dim": 16, "vocab_size": 3000}
    torch.manual_seed(0)
    hip = build_model(None, cfg).to(hip_device).train()
    b, _ = make_batch(3, 64, 3000)
    db = _to(b, hip_device)
    outs = []
    for _ in range(2):
        rep = torch.nn.parallel.replicate(hip, [hip_device.index or 0])[0]
        with torch.no_grad():
            outs.append(rep(db).cpu())
    assert not torch.equal(outs[0], outs[1])
    assert len(hip._rngs) == 1


# ---------------------------------------------------------------- device step bound
def test_device_step_bound_under_replay(hip_device):
    """A replayed hipGraph never passes through step()'s host guard.  Simulated by resetting the
    host counter: the device counter saturates at total_steps (schedule / coef_hist reads stay
    in bounds) and check_ids() raises OneCycleLR's ValueError."""
    V, B = 3000, 64
    htr = FiBiNETTrainer({"embedding_dim": 16, "vocab_size": V}, total_steps=2, batch_size=B, device=hip_device)
    for s in range(2):
        b, y = make_batch(s, B, V, device=hip_device)
        htr.step(b, y)
    htr.check_ids()
    assert htr.device_step() == 2
    htr.host_step = 0                                     # what a graph replay looks like to the host
    b, y = make_batch(9, B, V, device=hip_device)
    htr.step(b, y)
    assert htr.device_step() == 2
    with pytest.raises(ValueError):
        htr.check_ids()
