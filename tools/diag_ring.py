"""Diagnostics (GPU, one-rank RCCL): the sharded program-vs-eager lockstep of
tests/test_gpu_shard_program.py with the trainers' whole state compared after EVERY step, to find the
first step (and tensor) where they part.  FBN_RING_BF16 / the dtype / det from argv:
    python tools/diag_ring.py bf16 1 [same_last_next]"""
import ctypes
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("FBN_NATIVE_COMM", "1")


def main():
    dtype, det = sys.argv[1], sys.argv[2] == "1"
    same_last = len(sys.argv) > 3 and sys.argv[3] == "1"
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev, store=dist.HashStore())
    from ctr_recommendation_amd import _lib
    from ctr_recommendation_amd.data import make_batch
    from ctr_recommendation_amd.trainer import FC_CALIB_STEPS, FiBiNETTrainer
    from oracle.fibinet_oracle import build_model
    V, B, L = 60000, 1024, 20
    cfg = {"embedding_dim": 128, "vocab_size": V, "honour_config": True, "net_dropout": 0.0, "compute_dtype": dtype}
    torch.manual_seed(0)
    init = build_model(None, cfg, honour_config=True).state_dict()
    nb = 4
    bs = [make_batch(700 + s, B, V, device=dev) for s in range(nb + FC_CALIB_STEPS)]
    order = [nb + k for k in range(FC_CALIB_STEPS)] + [nb - 1] + list(range(nb)) * 5
    heavy_at = FC_CALIB_STEPS + 1 + 3 * nb
    total = len(order) + 4
    trs = [FiBiNETTrainer(cfg, total_steps=total, batch_size=B, device=dev,
                          init_state={k: v.clone() for k, v in init.items()}, shard=True, deterministic=det)
           for _ in range(2)]
    eager, prog_tr = trs
    print("ring", eager.ring.dtype, flush=True)
    pool = torch.cuda.MemPool()
    progs = {}
    names = ("E", "Em", "Ev", "row_state", "flat_p", "flat_m", "flat_v", "ring")
    for i, j in enumerate(order):
        if i == heavy_at:
            g = torch.Generator(device="cpu").manual_seed(99)
            full = torch.randint(1, V, (B, L), generator=g).to(dev)
            seq = bs[2][0]["item_seq"]
            src = (ctypes.c_void_p * 1)(full.data_ptr())
            dst = (ctypes.c_void_p * 1)(seq.data_ptr())
            nbytes = (ctypes.c_longlong * 1)(full.numel() * 8)
            _lib.call("fbn_copy_jobs", src, dst, nbytes, 1, _lib.stream_handle(dev))
            torch.cuda.synchronize()
        last = i + 1 == len(order)
        nxt = bs[order[i + 1]][0] if not last else (bs[0][0] if same_last else bs[order[0]][0])
        b, y = bs[j]
        le = eager.step(b, y, next_batch=nxt).item()
        if i < FC_CALIB_STEPS + 1:
            lp = prog_tr.step(b, y, next_batch=nxt).item()
            kind = "eager"
        elif j not in progs:
            progs[j] = prog_tr.record_program(b, y, next_batch=nxt, pool=pool)
            lp = prog_tr.loss.item()
            kind = "record"
        else:
            lp = prog_tr.run_program(progs[j]).item()
            kind = "replay"
        torch.cuda.synchronize()
        if os.environ.get("DIAG_FLUSH") == "1":
            for t in trs:
                t.flush()
            torch.cuda.synchronize()
        diff = [n for n in names if not torch.equal(getattr(eager, n), getattr(prog_tr, n))]
        diff.append(f"norm {eager.norm.item():.6g}/{prog_tr.norm.item():.6g} coef {eager.coef.item():.6g}")
        print(f"step {i:2d} batch {j} {kind:6s} loss {le:.7f} {lp:.7f} fc {eager.xchg.fc_active}/{prog_tr.xchg.fc_active} "
              f"differ: {diff}", flush=True)
    for t in trs:
        t.flush()
    torch.cuda.synchronize()
    print("after flush differ:", [n for n in names[:-1] if not torch.equal(getattr(eager, n), getattr(prog_tr, n))],
          flush=True)
    for t in trs:
        t.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
