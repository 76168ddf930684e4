"""CPU bisection of the training-run AUC gap -- TEST INFRASTRUCTURE.

    python -m tests.parity_bisect cpu [--perm-seed S] [--out ...json]     # oracle variants only
    python -m tests.parity_bisect hip --tag T [--nondet] --out T.npz      # one launcher run (GPU)
    python -m tests.parity_bisect report --hip a.npz,b.npz --out ...json  # oracle ensemble vs them

Runs the reference loop of tests/test_launcher.py::test_launcher_auc_parity_vs_reference_loop
(oracle Adam(L2) + BCE + clip + OneCycleLR over the restated BatchCollator, 2 epochs x 100 steps,
batch 512, d 16, dropout off, 5 000 items) in several numerically different but equally valid
variants, and one that emulates a candidate HIP deviation, then reports every variant's per-epoch
valid AUC and its distance (|dAUC|, max / mean |dp|) from the float64 loop:

* fp32 / f64: the oracle in float32 / float64 (the chaos floor of two correct implementations);
* fp32_t<n>: fp32 on n CPU threads (other reduction orders inside torch's kernels);
* fp32_foreach / fp32_fused: torch's multi-tensor / fused Adam (other operation orders of the step);
* f64_n<k> / fp32_n<k>: float64 (fp32) with relative 2^-24 noise (seed k) injected into every
  parameter after every step: an implementation that rounds like fp32 -- an independent trajectory
  of the chaos (the torch variants above share torch's kernels and stay correlated);
* fp32_g<k>: fp32 with gradient noise 10^-k x max |g| per tensor (does rounding-level gradient noise
  shift the learned AUC systematically?);
* fp32_fx40: the per-entry table-gradient vectors rounded to the 2^-40 fixed-point grid before the
  row sums -- what the deterministic duplicate fold (csrc/optim.hip sparse_fold_fx_kernel) did to
  every row several entries hit.
"""
from __future__ import annotations

import argparse
import json
import os
import tempfile
import time

import numpy as np
import torch

from ctr_recommendation_amd.data import write_microlens_parquet
from oracle.collate_ref import BatchCollatorRef, load_data
from oracle.fibinet_oracle import OracleFiBiNET, OracleTrainer, compute_auc


class _RoundGrad(torch.autograd.Function):
    """Identity forward; backward rounds the incoming gradient to a fixed-point grid of step 2^-shift."""

    @staticmethod
    def forward(ctx, x, shift):
        ctx.scale = float(2.0 ** shift)
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        s = ctx.scale
        return torch.round(g.double() * s).div(s).to(g.dtype), None


class _FxOracle(OracleFiBiNET):
    """The oracle with each table lookup's per-entry gradient rounded to 2^-shift."""

    shift = 40

    def fields(self, batch):
        emb = self.item_emb
        orig = emb.forward

        def fwd(idx):
            return _RoundGrad.apply(orig(idx), self.shift)
        emb.forward = fwd
        try:
            return super().fields(batch)
        finally:
            emb.forward = orig


def run_variant(name, data, perms, epochs, bs, n_train, n_valid):
    darray, coll, varray, vcoll = data
    f64 = name == "f64"
    cfg = {"embedding_dim": 16, "honour_config": True, "net_dropout": 0.0}
    nthreads = torch.get_num_threads()
    if name.startswith("fp32_t"):
        torch.set_num_threads(int(name[len("fp32_t"):]))
    try:
        torch.manual_seed(2025)
        cls = _FxOracle if name.startswith("fp32_fx") else OracleFiBiNET
        ref = cls(cfg, honour_config=True)
        if name.startswith("fp32_fx"):
            ref.shift = int(name[len("fp32_fx"):])
        if f64:
            ref = ref.double()
        gnoise = None
        if name.startswith("fp32_g"):
            # fp32 with relative gradient noise 10^-k of each tensor's max |g| injected before the
            # clip (diagnosis: does rounding-level gradient noise degrade the learned AUC?)
            gnoise = (float(10.0 ** -int(name[len("fp32_g"):])), torch.Generator().manual_seed(17))
        noise = None
        if name.startswith(("f64_n", "fp32_n")):
            # fp32-level rounding noise (relative 2^-24 x N(0,1), seed k) injected into every parameter
            # after every step, in float64 (an exact implementation that rounds like fp32) or fp32:
            # one more independent trajectory of the chaos every fp32 implementation goes through
            if name.startswith("f64_n"):
                ref = ref.double()
                f64 = True
            noise = torch.Generator().manual_seed(int(name.split("_n")[1]))
        cast = (lambda t: t.double() if t.is_floating_point() else t) if f64 else (lambda t: t)
        steps_per_epoch = -(-n_train // bs)
        otr = OracleTrainer(ref, lr=1e-3, weight_decay=1e-5, total_steps=epochs * steps_per_epoch)
        if gnoise is not None:
            amp, gen_ = gnoise

            def noisy_clip(params, max_norm, _orig=torch.nn.utils.clip_grad_norm_):
                params = list(params)
                with torch.no_grad():
                    for prm in params:
                        if prm.grad is not None:
                            prm.grad.add_(amp * prm.grad.abs().max() * torch.randn(prm.grad.shape, generator=gen_))
                return _orig(params, max_norm=max_norm)
            import oracle.fibinet_oracle as ofo
            ofo.torch.nn.utils.clip_grad_norm_ = noisy_clip
        if name in ("fp32_foreach", "fp32_fused"):
            otr.opt.param_groups[0]["foreach" if name == "fp32_foreach" else "fused"] = True
        aucs, losses, probs, steps = [], [], [], []
        for e in range(epochs):
            tot = 0.0
            for lo in range(0, n_train, bs):
                b, y = coll([darray[i, :] for i in perms[e][lo:lo + bs]])
                b = {k: cast(v.long() if k != "item_emb_d128" else v) for k, v in b.items()}
                ls = otr.step(b, cast(y))[0]
                if noise is not None:
                    with torch.no_grad():
                        for prm in ref.parameters():
                            prm.mul_((1.0 + 2.0 ** -24 * torch.randn(prm.shape, generator=noise,
                                                                     dtype=torch.float64)).to(prm.dtype))
                steps.append(ls)
                tot += ls
            losses.append(tot / steps_per_epoch)
            ref.eval()
            ys, ps = [], []
            with torch.no_grad():
                for lo in range(0, n_valid, bs):
                    b, y = vcoll([varray[i, :] for i in range(lo, min(n_valid, lo + bs))])
                    b = {k: cast(v.long() if k != "item_emb_d128" else v) for k, v in b.items()}
                    ps.append(ref(b).double().numpy())
                    ys.append(y.numpy())
            p = np.concatenate(ps)
            aucs.append(compute_auc(np.concatenate(ys), p))
            probs.append(p)
            ref.train()
    finally:
        torch.set_num_threads(nthreads)
        if gnoise is not None:
            import oracle.fibinet_oracle as ofo
            ofo.torch.nn.utils.clip_grad_norm_ = noisy_clip.__defaults__[0]
    return {"auc": aucs, "loss": losses, "probs": probs, "step_loss": steps,
            "sd": {k: v.detach().double().clone() for k, v in ref.state_dict().items()}}


ENSEMBLE = ("fp32", "fp32_t1", "fp32_t2", "fp32_fused", "f64_n1", "f64_n2", "f64_n3", "f64_n4")
BS, N_TRAIN, N_VALID, EPOCHS, N_ITEMS = 512, 51200, 8192, 2, 5000
PARITY_CONFIG = """
base_expid: MM_FiBiNET_Run
dataset_id: MicroLens_1M_x1
dataset_config:
  MicroLens_1M_x1:
    data_format: parquet
    train_data: {train}
    valid_data: {valid}
    item_info: {info}
MM_FiBiNET_Run:
  model: MM_FiBiNET
  learning_rate: 0.001
  batch_size: {bs}
  embedding_dim: 16
  max_len: 20
  epochs: {epochs}
  weight_decay: 1e-5
  seed: 2025
  honour_config: true
  net_dropout: 0.0
  deterministic: {det}
"""


def write_data(root):
    """The parity run's synthetic MicroLens-shaped parquet (train / valid / item_info)."""
    return write_microlens_parquet(os.path.join(root, "data"), n_train=N_TRAIN, n_valid=N_VALID, n_items=N_ITEMS,
                                   seed=77)


def oracle_data(p):
    darray, ci = load_data(p["train_data"])
    varray, vci = load_data(p["valid_data"])
    return darray, BatchCollatorRef(20, ci, p["item_info"]), varray, BatchCollatorRef(20, vci, p["item_info"])


def run_launcher(p, root, deterministic=True, noise_seed=0):
    """The launcher (python -m ctr_recommendation_amd.train) over the parity data on cuda:0:
    {"perms": the train loader's epoch permutations, "auc", "loss", "probs": final valid probabilities}.
    noise_seed k > 0: the HIP side of the ensemble -- after every step each trained parameter (the dense
    flat buffer and the item table) is multiplied by (1 + 2^-24 N(0,1)) in float64 and rounded back to
    fp32, as the oracle's f64_n<k> members are perturbed (device generator seeded k; test tooling,
    torch ops on the trainer's tensors between steps, nothing in the product path)."""
    from ctr_recommendation_amd.loader import ColumnarDataset, DeviceLoader, ItemInfoTable
    from ctr_recommendation_amd.train import load_config, run
    cfg_path = os.path.join(root, "fibinet_config.yaml")
    with open(cfg_path, "w") as f:
        f.write(PARITY_CONFIG.format(train=p["train_data"], valid=p["valid_data"], info=p["item_info"], bs=BS,
                                     epochs=EPOCHS, det=str(bool(deterministic)).lower()))
    drawn = []
    orig = DeviceLoader._perm

    def rec_perm(self):
        q = orig(self)
        if self.shuffle:
            drawn.append(q.cpu().numpy())
        return q
    DeviceLoader._perm = rec_perm
    from ctr_recommendation_amd.trainer import FiBiNETTrainer
    orig_step, step_loss = FiBiNETTrainer.step, []

    gen = None
    if noise_seed:
        gen = torch.Generator(device="cuda:0")
        gen.manual_seed(int(noise_seed))

    def rec_step(self, *a, **k):
        out = orig_step(self, *a, **k)
        step_loss.append(float(out.item()))
        if gen is not None:
            with torch.no_grad():
                for t in (self.flat_p, self.E):
                    f = 1.0 + 2.0 ** -24 * torch.randn(t.shape, generator=gen, device=t.device, dtype=torch.float64)
                    t.copy_((t.double() * f).to(t.dtype))
        return out
    FiBiNETTrainer.step = rec_step
    try:
        out = run(cfg_path, epochs=EPOCHS, checkpoint=os.path.join(root, "ck", "best.pth"), log=lambda *a, **k: None)
    finally:
        DeviceLoader._perm = orig
        FiBiNETTrainer.step = orig_step
    _, dcfg, _ = load_config(cfg_path)
    dev = torch.device("cuda", 0)
    vl = DeviceLoader(ColumnarDataset.from_parquet(dcfg["valid_data"], dev),
                      ItemInfoTable.from_parquet(dcfg["item_info"], dev), BS, shuffle=False)
    probs = np.concatenate([out["trainer"].predict(b).double().cpu().numpy() for b, _ in vl])
    hist = out["history"]
    return {"perms": drawn, "auc": [h[2] for h in hist], "loss": [h[1] for h in hist], "probs": probs,
            "trainer": out["trainer"], "step_loss": step_loss, "sd": out["trainer"].state_dict()}


def distances(r, base):
    """Per-epoch |dAUC| of r from base, and max / mean |dp| on the final valid probabilities."""
    pr = r["probs"][-1] if isinstance(r["probs"], list) else r["probs"]
    pb = base["probs"][-1] if isinstance(base["probs"], list) else base["probs"]
    return {"dAUC": [abs(a - b) for a, b in zip(r["auc"], base["auc"])],
            "max_abs_dp": float(np.abs(pr - pb).max()), "mean_abs_dp": float(np.abs(pr - pb).mean())}


LOSS_AT = (1, 2, 3, 5, 10, 20, 50, 100, 150, 200)


def trajectory(r, base):
    """|step loss - base step loss| at the steps LOSS_AT (1-based), and the final weights' distance
    from base's per tensor (relative Frobenius; BatchNorm buffers included)."""
    d = {f"step{s}": abs(r["step_loss"][s - 1] - base["step_loss"][s - 1]) for s in LOSS_AT
         if s <= len(r["step_loss"])}
    w = {}
    for k, v in base["sd"].items():
        if k in r["sd"] and v.is_floating_point() and k != "user_emb.weight":
            w[k] = float((r["sd"][k].double() - v).norm() / max(v.norm().item(), 1e-30))
    return {"step_loss_abs_diff": d, "weight_rel_dist": w}


def eval_weights(sd, data, f64=True):
    """AUC and probabilities of the given weights through the (float64) oracle's eval forward."""
    _, _, varray, vcoll = data
    cfg = {"embedding_dim": 16, "honour_config": True, "net_dropout": 0.0}
    m = OracleFiBiNET(cfg, honour_config=True)
    m.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in sd.items()})
    if f64:
        m = m.double()
    m.eval()
    ys, ps = [], []
    with torch.no_grad():
        for lo in range(0, N_VALID, BS):
            b, y = vcoll([varray[i, :] for i in range(lo, min(N_VALID, lo + BS))])
            b = {k: (v.double() if f64 and v.is_floating_point() else v) if k == "item_emb_d128" else v.long()
                 for k, v in b.items()}
            ps.append(m(b).double().numpy())
            ys.append(y.numpy())
    return compute_auc(np.concatenate(ys), np.concatenate(ps))


def first_step(p, data, seed=5):
    """One training step on the parity data's first batch (GPU): per tensor, the HIP trainer's
    gradient and update against the float64 oracle's, beside the fp32 oracle's distance from it.
    The step-2 loss of a HIP run sits ~50x further from the float64 loop than the fp32 loop's
    (tests/parity_bisect report: trajectory); this names the tensors whose first update differs."""
    from ctr_recommendation_amd.trainer import FiBiNETTrainer
    darray, coll, _, _ = data
    rows = np.random.default_rng(seed).permutation(N_TRAIN)[:BS]
    b, y = coll([darray[i, :] for i in rows])
    b = {k: (v.long() if k != "item_emb_d128" else v) for k, v in b.items()}
    cfg = {"embedding_dim": 16, "honour_config": True, "net_dropout": 0.0}
    torch.manual_seed(2025)
    init = OracleFiBiNET(cfg, honour_config=True).state_dict()
    res = {}
    for name in ("f64", "fp32"):
        m = OracleFiBiNET(cfg, honour_config=True)
        m.load_state_dict(init)
        cast = (lambda t: t.double() if t.is_floating_point() else t) if name == "f64" else (lambda t: t)
        if name == "f64":
            m = m.double()
        otr = OracleTrainer(m, lr=1e-3, weight_decay=1e-5, total_steps=EPOCHS * (N_TRAIN // BS))
        lr0 = otr.sched.get_last_lr()[0]
        otr.step({k: cast(v) for k, v in b.items()}, cast(y))
        res[name] = {"g": {n: q.grad.detach().double().clone() for n, q in m.named_parameters() if q.grad is not None},
                     "sd": {k: v.detach().double().clone() for k, v in m.state_dict().items()}, "norm": otr.last_total_norm}
    dev = torch.device("cuda", 0)
    htr = FiBiNETTrainer(dict(cfg, deterministic=True), total_steps=EPOCHS * (N_TRAIN // BS), batch_size=BS,
                         device=dev, init_state={k: v.clone() for k, v in init.items()})
    htr.step({k: v.to(dev) for k, v in b.items()}, y.to(dev))
    torch.cuda.synchronize()
    res["hip"] = {"g": {n: t.detach().double().cpu() for n, t in htr.g.items()},
                  "sd": {k: v.double() for k, v in htr.state_dict().items()}, "norm": float(htr.norm.item())}
    out = {"lr0": lr0, "clip_norm": {k: r["norm"] for k, r in res.items()}, "tensors": {}}
    ref = res["f64"]
    for n, v in ref["sd"].items():
        if not v.is_floating_point() or n == "user_emb.weight":
            continue
        ent = {}
        for who in ("fp32", "hip"):
            d_ref = v - init[n].double()
            d_who = res[who]["sd"][n] - init[n].double()
            dd = (d_who - d_ref).abs()
            ent[who] = {"update_max_abs_diff_over_lr": float(dd.max() / lr0),
                        "elements_off_by_1pct_lr": int((dd > 0.01 * lr0).sum()), "numel": v.numel()}
            if n in ref["g"] and n in res[who]["g"]:
                gr, gw = ref["g"][n], res[who]["g"][n].reshape(ref["g"][n].shape)
                ent[who]["grad_max_abs_diff_over_max"] = float((gw - gr).abs().max() / max(gr.abs().max(), 1e-30))
        out["tensors"][n] = ent
    return out


def ensemble(data, perms, names=("f64",) + ENSEMBLE):
    return {n: run_variant(n, data, perms, EPOCHS, BS, N_TRAIN, N_VALID) for n in names}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("cpu", "hip", "report", "step1"))
    ap.add_argument("--out", default=None)
    ap.add_argument("--variants", default="f64,fp32,fp32_t1,fp32_t2,fp32_fused,f64_n1,f64_n2,f64_n3,f64_n4,fp32_fx40,fp32_g6")
    ap.add_argument("--perm-seed", type=int, default=5)
    ap.add_argument("--tag", default="default")
    ap.add_argument("--nondet", action="store_true")
    ap.add_argument("--hip", default="", help="report: comma-separated npz files of hip runs")
    args = ap.parse_args(argv)
    root = tempfile.mkdtemp()
    p = write_data(root)
    data = oracle_data(p)
    if args.mode == "step1":
        out = first_step(p, data)
        print(json.dumps(out, indent=1))
        if args.out:
            with open(args.out, "w") as f:
                json.dump(out, f, indent=1)
        return
    if args.mode == "hip":
        # one launcher run (the library FBN_LIB_PATH names) -> npz for the report
        r = run_launcher(p, root, deterministic=not args.nondet)
        np.savez(args.out, perms=np.stack(r["perms"]), auc=np.array(r["auc"]), loss=np.array(r["loss"]),
                 probs=r["probs"], tag=args.tag, lib=os.environ.get("FBN_LIB_PATH", "libfibinet_hip.so"),
                 step_loss=np.array(r["step_loss"]))
        torch.save(r["sd"], args.out[:-4] + ".pt")
        print(f"hip {args.tag}: auc {r['auc']} loss {r['loss']}", flush=True)
        return
    if args.mode == "cpu":
        rng = np.random.default_rng(args.perm_seed)
        perms = [rng.permutation(N_TRAIN) for _ in range(EPOCHS)]
        hips = {}
        names = args.variants.split(",")
    else:
        hips = {}
        for f in args.hip.split(","):
            z = np.load(f, allow_pickle=False)
            hips[str(z["tag"])] = {"perms": list(z["perms"]), "auc": list(z["auc"]), "loss": list(z["loss"]),
                                   "probs": z["probs"], "lib": str(z["lib"]), "step_loss": list(z["step_loss"]),
                                   "sd": {k: v.double() for k, v in
                                          torch.load(f[:-4] + ".pt", weights_only=True).items()}}
        perms = next(iter(hips.values()))["perms"]
        for h in hips.values():
            assert all((a == b).all() for a, b in zip(h["perms"], perms)), "hip runs drew different permutations"
        names = args.variants.split(",")
    res = {}
    for name in names:
        t0 = time.time()
        res[name] = run_variant(name, data, perms, EPOCHS, BS, N_TRAIN, N_VALID)
        print(f"{name}: auc {res[name]['auc']} loss {res[name]['loss']} ({time.time() - t0:.0f} s)", flush=True)
    base = res["f64"]
    rec = {"run": f"{EPOCHS} epochs x {N_TRAIN // BS} steps, batch {BS}, d 16, {N_ITEMS} items, dropout off, "
                  + (f"perm seed {args.perm_seed}" if args.mode == "cpu" else "the launcher's permutations"),
           "oracle": {}, "hip": {}}
    for name, r in res.items():
        rec["oracle"][name] = {"auc": r["auc"], "train_loss": r["loss"]}
        if name != "f64":
            rec["oracle"][name]["vs_f64"] = distances(r, base)
    ens = [n for n in ENSEMBLE if n in res]
    if ens:
        floor = [max(rec["oracle"][n]["vs_f64"]["dAUC"][e] for n in ens) for e in range(EPOCHS)]
        rec["ensemble"] = {"members": ens, "max_dAUC_vs_f64": floor,
                           "gate": [max(1e-4, 2 * f) for f in floor],
                           "max_abs_dp_vs_f64": max(rec["oracle"][n]["vs_f64"]["max_abs_dp"] for n in ens),
                           "mean_abs_dp_vs_f64": max(rec["oracle"][n]["vs_f64"]["mean_abs_dp"] for n in ens)}
    for name, r in res.items():
        if name != "f64":
            rec["oracle"][name]["trajectory_vs_f64"] = trajectory(r, base)
    for tag, h in hips.items():
        rec["hip"][tag] = {"lib": h["lib"], "auc": h["auc"], "train_loss": h["loss"], "vs_f64": distances(h, base),
                           "vs_fp32": distances(h, res["fp32"]) if "fp32" in res else None,
                           "trajectory_vs_f64": trajectory(h, base),
                           "final_weights_through_f64_oracle_forward_auc": eval_weights(h["sd"], data)}
    tags = list(hips)
    for i in range(len(tags)):
        for j in range(i + 1, len(tags)):
            rec["hip"][f"{tags[i]}_vs_{tags[j]}"] = distances(hips[tags[i]], hips[tags[j]])
    print(json.dumps(rec, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
