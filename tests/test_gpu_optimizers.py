"""Opt-in optimizer variants, pytest -m gpu.

* AdamW (the config's ``optimizer: adamw``, config/fibinet_config.yaml:62, which the reference's
  code ignores -- src/train_fibinet.py:78 uses Adam): native trainer vs torch.optim.AdamW on the
  oracle, and its lazy table replay bit-identical to the eager table pass;
* sparse table Adam (table_adam="sparse", for 100M-row tables): only touched rows move, as
  torch.optim.SparseAdam; vs the oracle's sparse rule.
Bars as test_gpu_trainer: loss 2e-5 at step 0 and 5e-4 after; eval probabilities 2e-3.
"""
import pytest
import torch

from ctr_recommendation_amd.data import make_batch
from ctr_recommendation_amd.trainer import FiBiNETTrainer
from oracle.fibinet_oracle import OracleTrainer, build_model as oracle_build

pytestmark = pytest.mark.gpu
NO_DROP = {"honour_config": True, "net_dropout": 0.0}


def _to(b, dev):
    return {k: v.to(dev) for k, v in b.items()}


@pytest.mark.parametrize("variant", [dict(optimizer="adamw"), dict(table_adam="sparse"),
                                     dict(optimizer="adamw", table_adam="sparse")])
@pytest.mark.parametrize("d", [16, 128])
def test_optimizer_variant_matches_oracle(hip_device, d, variant):
    V, B, total = 3000, 256, 40
    cfg = dict({"embedding_dim": d, "vocab_size": V}, **NO_DROP)
    torch.manual_seed(0)
    ref = oracle_build(None, cfg, honour_config=True)
    init = {k: v.clone() for k, v in ref.state_dict().items()}
    otr = OracleTrainer(ref, lr=1e-3, weight_decay=1e-2, total_steps=total,      # wd 1e-2: the decay is visible
                        optimizer=variant.get("optimizer", "adam"),
                        table_optimizer="sparse" if variant.get("table_adam") == "sparse" else "dense")
    htr = FiBiNETTrainer(cfg, total_steps=total, batch_size=B, device=hip_device, weight_decay=1e-2,
                         init_state={k: v.clone() for k, v in init.items()}, lazy_window=4, **variant)
    touched = torch.zeros(V, dtype=torch.bool)
    for s in range(5):
        b, y = make_batch(900 + s, B, V)
        touched[b["item_id"]] = True
        touched[b["item_seq"].flatten()] = True
        lh = htr.step(_to(b, hip_device), y.to(hip_device)).item()
        lr_, _ = otr.step(b, y)
        assert abs(lh - lr_) < (2e-5 if s == 0 else 5e-4), (s, lh, lr_)
    htr.check_ids()
    E = htr.state_dict()["item_emb.weight"]
    touched[0] = False
    if variant.get("table_adam") == "sparse":
        # untouched rows never move
        assert torch.equal(E[~touched], init["item_emb.weight"][~touched])
    else:
        assert not torch.equal(E[~touched][1:], init["item_emb.weight"][~touched][1:])
    assert (E - ref.item_emb.weight.detach()).abs().max().item() < 2e-3 * 10    # a few lr-sized steps
    b, _ = make_batch(999, 512, V)
    ref.eval()
    with torch.no_grad():
        pr = ref(b)
    ph = htr.predict(_to(b, hip_device)).cpu()
    assert (pr - ph).abs().max().item() < 2e-3


def test_adamw_lazy_replay_bit_identical_to_eager(hip_device):
    """The AdamW zero-gradient replay (decoupled decay in the catch-up) == the eager table pass."""
    V, B, d = 5000, 128, 128
    cfg = {"embedding_dim": d, "vocab_size": V}
    torch.manual_seed(0)
    init = oracle_build(None, cfg).state_dict()
    kw = dict(total_steps=20, batch_size=B, device=hip_device, init_state=init, optimizer="adamw", weight_decay=1e-2)
    eager = FiBiNETTrainer(cfg, table_adam="eager", **kw)
    lazy = FiBiNETTrainer(cfg, table_adam="lazy", lazy_window=4, **kw)
    for s in range(8):
        b, y = make_batch(70 + s, B, V)
        db = _to(b, hip_device)
        eager.step(db, y.to(hip_device))
        lazy.step(db, y.to(hip_device))
    lazy.flush()
    torch.cuda.synchronize()
    # rows no batch touched took only zero-gradient steps: bit-identical
    touched = torch.zeros(V, dtype=torch.bool, device=hip_device)
    for s in range(8):
        b, _ = make_batch(70 + s, B, V)
        touched[b["item_id"].to(hip_device)] = True
        touched[b["item_seq"].flatten().to(hip_device)] = True
    un = ~touched
    assert torch.equal(eager.E[un], lazy.E[un])
    assert torch.equal(eager.Em[un], lazy.Em[un]) and torch.equal(eager.Ev[un], lazy.Ev[un])
