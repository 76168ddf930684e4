"""Step programs (the native step driver, csrc/plan.cpp): a recorded training step replayed by one
host call must be bit-identical to running the step eagerly (src/train_fibinet.py:113-123's loop
body), in every mode the bench times -- bf16 at d 128 (two streams, the next-batch prefetch, the
duplicate fold on the side stream), fp32 at d 128 (per-step temporaries from the program's private
memory pool), d 16 (the side passes in sequence on the main stream) -- and when replays interleave
with eager steps (the bench's probe steps run eagerly between replays)."""
import pytest
import torch

from ctr_recommendation_amd.data import make_batch
from ctr_recommendation_amd.trainer import FiBiNETTrainer
from oracle.fibinet_oracle import build_model as oracle_build

pytestmark = pytest.mark.gpu


def _trainer(cfg, init, B, dev):
    return FiBiNETTrainer(cfg, total_steps=60, batch_size=B, device=dev,
                          init_state={k: v.clone() for k, v in init.items()})


@pytest.mark.parametrize("d,dtype", [(128, "bf16"), (128, "fp32"), (16, "fp32"), (128, "bf16_fwd")])
def test_program_replay_bit_identical_to_eager(hip_device, d, dtype):
    V, B, nb, steps = 40000, 512, 4, 14
    cfg = {"embedding_dim": d, "vocab_size": V, "compute_dtype": dtype}
    torch.manual_seed(0)
    init = oracle_build(None, dict(cfg, honour_config=False)).state_dict()
    batches = []
    for j in range(nb):
        b, y = make_batch(60 + j, B, V)
        batches.append(({k: v.to(hip_device) for k, v in b.items()}, y.to(hip_device)))
    eager = _trainer(cfg, init, B, hip_device)
    prog_tr = _trainer(cfg, init, B, hip_device)
    progs = {}
    le, lp = [], []
    # one step ahead of the first recording that prefetches (and pre-claims) its batch, as a replay
    # of program 0 will always follow one (program 3's step).  Its own claims have no pre-claims
    # (compare-and-swap: with repeated ids the winning entry is timing-dependent), so its batch has
    # every id once: both trainers start from the same bits
    wb, wy = make_batch(59, B, V)
    L = wb["item_seq"].shape[1]
    ids = torch.randperm(V - 1, generator=torch.Generator().manual_seed(5))[:B * (L + 1)].view(B, L + 1) + 1
    wb["item_id"] = ids[:, 0].clone()
    wb["item_seq"] = torch.where(wb["item_seq"] > 0, ids[:, 1:], torch.zeros_like(ids[:, 1:]))
    wb, wy = {k: v.to(hip_device) for k, v in wb.items()}, wy.to(hip_device)
    for tr in (eager, prog_tr):
        tr.step(wb, wy, next_batch=batches[0][0])
    for i in range(steps):
        b, y = batches[i % nb]
        nxt = batches[(i + 1) % nb][0]
        le.append(eager.step(b, y, next_batch=nxt).item())
        j = i % nb
        if j not in progs:
            progs[j] = prog_tr.record_program(b, y, next_batch=nxt)      # a real step, recorded
        elif i == 9:
            prog_tr.step(b, y, next_batch=nxt)                           # an eager step between replays
        else:
            prog_tr.run_program(progs[j])
        lp.append(prog_tr.loss.item())
    assert le == lp, (le, lp)
    assert prog_tr.device_step() == eager.device_step() == steps + 1
    eager.flush()
    prog_tr.flush()
    for name in ("E", "Em", "Ev", "flat_p", "flat_m", "flat_v"):
        assert torch.equal(getattr(eager, name), getattr(prog_tr, name)), name
    for k in ("mlp.1.running_mean", "mlp.1.running_var", "mlp.5.running_mean", "mlp.5.num_batches_tracked"):
        assert torch.equal(eager.p[k], prog_tr.p[k]), k
    assert all(len(p) > 10 for p in progs.values())
    # out of the recorded order (the previous step prefetched another batch): refused
    with pytest.raises(RuntimeError, match="out of order"):
        prog_tr.run_program(progs[(steps + 1) % nb])


def test_program_refuses_unsupported_paths(hip_device):
    cfg = {"embedding_dim": 16, "vocab_size": 3000}
    torch.manual_seed(0)
    tr = FiBiNETTrainer(cfg, total_steps=10, batch_size=64, device=hip_device, table_adam="eager")
    b, y = make_batch(1, 64, 3000)
    with pytest.raises(ValueError, match="lazy table Adam"):
        tr.record_program({k: v.to(hip_device) for k, v in b.items()}, y.to(hip_device))
