"""Diagnostics: eager vs program sharded trainers (one-rank RCCL job), per step the loss, the
fold's extra buffer at rest (must be zero) and the table difference.  GPU box only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29613", FBN_NATIVE_COMM="1")
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
from ctr_recommendation_amd.data import make_batch
from ctr_recommendation_amd.trainer import FC_CALIB_STEPS, FiBiNETTrainer
from oracle.fibinet_oracle import build_model

V, B, L = 60000, 1024, 20
dtype = os.environ.get("DTYPE", "bf16")
cfg = {"embedding_dim": 128, "vocab_size": V, "honour_config": True, "net_dropout": 0.0, "compute_dtype": dtype}
torch.manual_seed(0)
init = build_model(None, cfg, honour_config=True).state_dict()
nb = 4
bs = [make_batch(700 + s, B, V, device=dev) for s in range(nb + FC_CALIB_STEPS)]
order = [nb + k for k in range(FC_CALIB_STEPS)] + [nb - 1] + list(range(nb)) * 3
trs = [FiBiNETTrainer(cfg, total_steps=len(order) + 4, batch_size=B, device=dev,
                      init_state={k: v.clone() for k, v in init.items()}, shard=True) for _ in range(2)]
eager, pt = trs
pool = torch.cuda.MemPool()
progs = {}


def ex(t):
    return float(t._fc_extra.abs().max()) if t._fc_extra is not None else -1.0


for i, j in enumerate(order):
    nxt = bs[order[i + 1]][0] if i + 1 < len(order) else bs[order[0]][0]
    b, y = bs[j]
    le = eager.step(b, y, next_batch=nxt).item()
    if i < FC_CALIB_STEPS + 1:
        lp = pt.step(b, y, next_batch=nxt).item()
        kind = "step"
    elif j not in progs:
        progs[j] = pt.record_program(b, y, next_batch=nxt, pool=pool)
        lp = pt.loss.item()
        kind = "record"
    else:
        lp = pt.run_program(progs[j]).item()
        kind = "replay"
    torch.cuda.synchronize()
    dE = float((eager.E - pt.E).abs().max())
    nrows = int(((eager.E - pt.E).abs().amax(1) > 1e-6).sum())
    dp = float((eager.flat_p - pt.flat_p).abs().max())
    print(f"{i:2d} b{j} {kind:6s} loss {le:.6f}/{lp:.6f} extra {ex(eager):.3g}/{ex(pt):.3g} "
          f"slotflag {int((eager.slot_row != -1).sum())}/{int((pt.slot_row != -1).sum())} "
          f"map {int((eager.map != -1).sum())}/{int((pt.map != -1).sum())} dE {dE:.3g} rows {nrows} dp {dp:.3g} "
          f"step {int(eager.step_dev[0]) if eager.step_dev.numel() else -1}/{int(pt.step_dev[0])} "
          f"fc {eager.xchg.fc_active}/{pt.xchg.fc_active}", flush=True)
    if kind == "replay" and ex(pt) > 0 and not globals().get("_shown"):
        _shown = True
        ids = pt.xchg.fc_set["recv_ids"].cpu()
        nzu = (pt._fc_extra.abs().amax(1) > 0).nonzero().flatten().cpu()
        print("residue entries", nzu.numel(), "of", ids.numel(), "cap", pt.xchg.cap, flush=True)
        first = {}
        cnt = {}
        for e, r in enumerate(ids.tolist()):
            if r < 0 or r == 0:
                continue
            first.setdefault(r, e)
            cnt[r] = cnt.get(r, 0) + 1
        for u in nzu[:12].tolist():
            r = int(ids[u])
            print(f"  u {u} id {r} first {first.get(r)} count {cnt.get(r)} extra_norm {float(pt._fc_extra[u].norm()):.3g}",
                  flush=True)
        nclaim = sum(1 for u in nzu.tolist() if int(ids[u]) > 0 and first.get(int(ids[u])) == u)
        print("  residue at true first entries:", nclaim, "dup rows total:", sum(1 for c in cnt.values() if c > 1),
              flush=True)
for t in trs:
    t.close()
dist.destroy_process_group()
