"""End-to-end training throughput at C3: batches assembled in HBM by the device collator each step.

bench.py times the train step on pre-built HBM-resident batches (SURVEY §8's hot path).  This
times what a user of the launcher gets: every step first collates its batch from the columnar
dataset (fbn_collate: row gather of the id / level / label columns, the last max_len history ids,
the item_id -> item_emb_d128 lookup in the HBM item_info table -- src/dataloader.py:53-121's
BatchCollator), then runs the trainer's step, shuffled epoch order, N = 1, eager (the batch
buffers are new every step, so no graph replay).  The collation of step i + 1 is issued before
step i so that step i can catch the next batch's rows up ahead (next_batch), as the launcher does.

Synthetic MicroLens-shaped data: 160 batches of interactions over 1.25 M items (ids ~ U[1, V)),
history lengths ~ U{0..20} stored 24 wide (left-padded), item_info fp32 [V, 128].
Prints one JSON line.  Usage (GPU box): python tools/bench_e2e.py [--steps K] [--dtype bf16]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def synthetic_columns(n, V, Ls, seed=2025):
    rng = np.random.default_rng(seed)
    n_valid = rng.integers(0, 21, n)
    seq = rng.integers(1, V, (n, Ls), dtype=np.int64)
    seq[np.arange(Ls)[None, :] < (Ls - n_valid)[:, None]] = 0          # left padding
    return {"item_id": rng.integers(1, V, n, dtype=np.int64), "item_seq": seq,
            "likes_level": rng.integers(0, 11, n, dtype=np.int64), "views_level": rng.integers(0, 11, n, dtype=np.int64),
            "user_id": rng.integers(1, 1 << 20, n, dtype=np.int64), "label": rng.integers(0, 2, n).astype(np.float32)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--rows", type=int, default=1_250_000)
    ap.add_argument("--batches", type=int, default=160)
    ap.add_argument("--dtype", default="bf16")
    args = ap.parse_args()
    from bench import _initial_state
    from ctr_recommendation_amd.loader import ColumnarDataset, DeviceLoader, ItemInfoTable
    from ctr_recommendation_amd.trainer import FiBiNETTrainer

    dev = torch.device("cuda", 0)
    B, V, d, F = args.batch, args.rows, 128, 128
    cfg = {"embedding_dim": d, "vocab_size": V, "compute_dtype": args.dtype}
    ds = ColumnarDataset(synthetic_columns(B * args.batches, V, 24), dev)
    g = np.random.default_rng(7)
    info = ItemInfoTable(np.arange(V, dtype=np.int64), g.standard_normal((V, 128), dtype=np.float32), dev)
    loader = DeviceLoader(ds, info, B, shuffle=True, max_len=20, drop_last=True)
    prime = 2 * F
    total = prime + args.steps + 8
    tr = FiBiNETTrainer(cfg, total_steps=total, batch_size=B, device=dev, init_state=_initial_state(cfg, V, 1, 0, dev),
                        lazy_window=F)

    def batches():
        while True:
            yield from loader

    it = batches()
    cur = next(it)

    def run(n):
        nonlocal cur
        for _ in range(n):
            nxt = next(it)                      # collate the next batch (device), then step this one
            tr.step(cur[0], cur[1], next_batch=nxt[0])
            cur = nxt

    run(prime)                                  # lazy table Adam to steady state (as bench.py)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    loader.check()
    tr.check_ids()

    # the collation alone: one fbn_collate launch per batch, HIP events on the current stream
    perm = torch.randperm(len(ds), device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(20_000_000)
    e0.record()
    nc = 50
    for i in range(nc):
        loader.collate(perm[(i % args.batches) * B:((i % args.batches) + 1) * B])
    e1.record()
    torch.cuda.synchronize()
    coll_ms = e0.elapsed_time(e1) / nc
    # algorithmic bytes of one collation: per sample the row index, 5 scalar columns read + written,
    # max_len history ids read + written, the item_info slot (4 B) and its 128-float row + written copy
    per_sample = 8 + 5 * 8 * 2 + 20 * 8 * 2 + 4 + 128 * 4 * 2
    print(json.dumps({
        "metric": "end-to-end training samples/sec (device collator + full train step)", "unit": "samples/s",
        "value": round(B * args.steps / dt, 1), "ms_per_step": round(dt / args.steps * 1e3, 4), "steps": args.steps,
        "priming_steps": prime, "dtype": args.dtype, "n_gpus": 1,
        "collate": {"avg_launch_ms": round(coll_ms, 4), "bytes_per_launch": per_sample * B,
                    "achieved_GBps": round(per_sample * B / (coll_ms * 1e-3) / 1e9, 1)},
        "config": {"workload": "C3 via the HBM-resident loader: d=128 + item_emb_d128, batch 8192, history 20 "
                               "(stored 24 wide), 1.25 M items, shuffled epochs of 160 batches",
                   "graph": False},
        "data": "synthetic MicroLens-shaped columnar dataset + item_info table, HBM-resident",
        "final_loss": round(float(tr.loss.item()), 5)}), flush=True)


if __name__ == "__main__":
    main()
