"""Config C5's per-GPU shard on one MI355X: 100 M item rows over 8 GPUs = 12.5 M rows x d 128 per
GPU (src/model_fibinet.py:100 at that vocabulary; the reference's dense Adam over the whole table,
src/train_fibinet.py:78,121, is what the lazy replay stands in for).

* the memory plan holds: table + Adam moments (3 x 6.4 GB), the deferred-gradient ring and the
  tagged pre-claims allocate and run at B = 8192, history 20;
* lazy table Adam (claims, next-batch prefetch, rolling window of V / F = 97.7 K rows per step,
  deferred gradients, flush) is bit-identical to the eager pass over all 12.5 M rows each step --
  table, both moments, dense parameters and losses (duplicates folded by the deterministic
  fixed-point sums in both runs, so no float-atomic order enters);
* id bounds at this size: the largest id (V - 1) is gathered and updated, an id of V raises
  IndexError at check_ids();
* the opt-in sparse table Adam (the C5 variant) runs the same steps (touched rows only).
"""
import pytest
import torch

from ctr_recommendation_amd.data import make_device_batches
from ctr_recommendation_amd.model_fibinet import build_model
from ctr_recommendation_amd.trainer import FiBiNETTrainer

pytestmark = pytest.mark.gpu
V, D, B, L, STEPS = 12_500_000, 128, 8192, 20, 4


def _init(dev):
    torch.manual_seed(0)
    init = dict(build_model(None, {"embedding_dim": D, "vocab_size": 4}).state_dict())
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    table = torch.randn((V, D), generator=g, device=dev)
    table[0].zero_()
    return init, table


def test_c5_shard_lazy_equals_eager(hip_device):
    init, table = _init(hip_device)
    cfg = {"embedding_dim": D, "vocab_size": V}
    batches = make_device_batches(STEPS + 1, B, V, L, hip_device, seed=77)
    batches[0][0]["item_id"][0] = V - 1                    # the last row of the shard
    batches[1][0]["item_seq"][3, -1] = V - 1
    runs = {}
    for mode in ("eager", "lazy"):
        tr = FiBiNETTrainer(cfg, total_steps=20, batch_size=B, device=hip_device,
                            init_state=dict(init, **{"item_emb.weight": table.clone()}), table_adam=mode,
                            deterministic=True)
        losses = []
        for s in range(STEPS):
            b, y = batches[s]
            losses.append(tr.step(b, y, next_batch=batches[s + 1][0] if mode == "lazy" else None).item())
        tr.check_ids()
        tr.flush()
        torch.cuda.synchronize()
        runs[mode] = tr, losses
    (te, le), (tl, ll) = runs["eager"], runs["lazy"]
    assert le == ll, (le, ll)
    assert torch.equal(te.flat_p, tl.flat_p)
    for a, c in ((te.E, tl.E), (te.Em, tl.Em), (te.Ev, tl.Ev)):
        assert torch.equal(a, c)
    assert int(tl.last.min()) == STEPS and int(tl.last.max()) == STEPS     # every row current after flush
    assert bool((tl.E[V - 1] != table[V - 1]).any())                          # the last row was updated
    del runs, te, tl
    # the opt-in sparse table Adam on the same shard (touched rows only; untouched rows keep their
    # init and zero moments)
    tr = FiBiNETTrainer(cfg, total_steps=20, batch_size=B, device=hip_device,
                        init_state=dict(init, **{"item_emb.weight": table.clone()}), table_adam="sparse")
    for s in range(STEPS):
        b, y = batches[s]
        loss = tr.step(b, y).item()
        assert loss == loss and loss > 0
    torch.cuda.synchronize()
    ids = torch.cat([batches[s][0]["item_id"] for s in range(STEPS)] +
                    [batches[s][0]["item_seq"].flatten() for s in range(STEPS)])
    touched = torch.zeros(V, dtype=torch.bool, device=hip_device)
    touched[ids] = True
    touched[0] = False
    assert torch.equal(tr.E[~touched], table[~touched])
    assert bool((tr.Em[touched] != 0).any(1).all())
    # an id past the shard raises what nn.Embedding raises
    bad = {k: v.clone() for k, v in batches[STEPS][0].items()}
    bad["item_id"][5] = V
    tr.predict(bad)
    with pytest.raises(IndexError):
        tr.check_ids()
