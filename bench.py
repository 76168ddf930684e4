"""Benchmark: FiBiNET training samples/s on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Workload (DESIGN.md "Benchmark"): config C3 of BASELINE.json -- FiBiNET emb_dim=128 with the
item_emb_d128 dense feature, batch 8192 per GPU, history 20, bf16 GEMM operands / fp32
accumulation and fp32 master weights, full training step (fwd + BCE + bwd + clip + Adam(L2) +
OneCycleLR), synthetic MicroLens-shaped batches resident in HBM.  Item vocabulary: 1.25 M rows
per GPU, row-sharded (N = 8 -> the 10 M rows of config C4).  Weak scaling: per-GPU batch and
per-GPU table shard are fixed as N grows.

One JSON line on rank 0 with the contract keys plus
  roofline:      the dominant kernel (dense Adam over the table shard), HIP events around its
                 launches inside the probe pass (same stream), algorithmic bytes per launch;
  roofline_gather: the fused embedding gather (fields_fwd) with SURVEY §8(d)'s 12,984 B/sample;
  cpu_baseline:  the oracle's torch-CPU restatement of the reference train step (rank 0, N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
ROWS_PER_GPU = 1_250_000


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8192, help="per-GPU batch")
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--rows-per-gpu", type=int, default=ROWS_PER_GPU)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=6)
    ap.add_argument("--probe-steps", type=int, default=10)
    return ap.parse_args()


def gather_bytes_per_sample(d: int, L: int = 20) -> int:
    # (L+1) rows requested + 23 int64 ids + 4 output rows (item, hist, likes, views)
    return (L + 1) * d * 4 + (L + 3) * 8 + 4 * d * 4


def adam_table_bytes(rows: int, d: int, touched: int) -> int:
    # read+write p, m, v (24 B/elem) + the row->slot map (4 B/row) + the touched gradient rows
    return 24 * rows * d + 4 * rows + 4 * touched * d


def cpu_baseline(args, world):
    """Oracle (torch CPU restatement of train_fibinet.py's step) on this host's cores."""
    from ctr_recommendation_amd.data import make_batch
    from oracle.fibinet_oracle import OracleTrainer, build_model
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    threads = max(1, min(threads, len(os.sched_getaffinity(0))))
    torch.set_num_threads(threads)
    d, B, V = args.dim, args.batch, args.rows_per_gpu
    torch.manual_seed(2025)
    model = build_model(None, {"embedding_dim": d, "vocab_size": V})
    tr = OracleTrainer(model, lr=1e-3, weight_decay=1e-5, total_steps=1000)
    batches = [make_batch(7 + i, B, V) for i in range(2)]
    tr.step(*batches[0])                      # warm-up (allocations, Adam state)
    n = args.cpu_steps
    t0 = time.perf_counter()
    for i in range(n):
        tr.step(*batches[i % 2])
    dt = time.perf_counter() - t0
    return {"value": round(n * B / dt, 2), "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"{n} timed steps (+1 warm-up) of the oracle train step (torch {torch.__version__} CPU, "
                      f"fp32) at d={d}, batch {B}, {V} item rows, history 20 -- the same per-GPU workload"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    group = None
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    from ctr_recommendation_amd.data import make_device_batches
    from ctr_recommendation_amd.trainer import FiBiNETTrainer

    d, B, L = args.dim, args.batch, 20
    V = args.rows_per_gpu * world
    cfg = {"embedding_dim": d, "vocab_size": V, "compute_dtype": args.dtype}
    K, W = args.steps, args.warmup
    total = W + K + args.probe_steps + 16
    # initial table: N(0,1) rows like nn.Embedding (row 0 = padding = 0), built on the device
    torch.manual_seed(2025)
    from ctr_recommendation_amd.model_fibinet import build_model
    small = build_model(None, dict(cfg, vocab_size=4)).state_dict()
    init = {k: v for k, v in small.items()}
    g = torch.Generator(device=dev)
    g.manual_seed(2025)
    lo = rank * ((V + world - 1) // world)
    table = torch.randn((V if world == 1 else 1, d), generator=g, device=dev) if world == 1 else None
    if world == 1:
        table[0].zero_()
        init["item_emb.weight"] = table
    else:
        # each rank only materialises its own shard; the trainer slices init[...][lo:hi]
        class _Shard:
            shape = (V, d)

            def __getitem__(self, sl):
                n = min(V, sl.stop) - sl.start
                t = torch.randn((n, d), generator=g, device=dev)
                if sl.start == 0:
                    t[0].zero_()
                return t
        init["item_emb.weight"] = _Shard()
    tr = FiBiNETTrainer(cfg, total_steps=total, batch_size=B, device=dev, rank=rank, world=world,
                        init_state=init)
    del table
    batches = make_device_batches(4, B, V, L, dev, seed=2025 + rank)
    # static inputs for graph replay
    sb = {k: v.clone() for k, v in batches[0][0].items()}
    sl = batches[0][1].clone()

    def load(i):
        b, y = batches[i % len(batches)]
        for k in sb:
            sb[k].copy_(b[k], non_blocking=True)
        sl.copy_(y, non_blocking=True)

    use_graph = world == 1 and not args.no_graph
    for i in range(W):
        load(i)
        tr.step(sb, sl)
    graphs = []
    if use_graph:
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            tr.step(*batches[0])                  # side-stream warm-up required before capture
        torch.cuda.current_stream().wait_stream(s)
        # one graph per HBM-resident batch (shared memory pool): the timed loop is pure replays
        pool = None
        for b, y in batches:
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, pool=pool):
                tr.step(b, y)
            pool = gr.pool()
            graphs.append(gr)
        torch.cuda.synchronize()

    def run_step(i):
        if graphs:
            graphs[i % len(graphs)].replay()
        else:
            load(i)
            tr.step(sb, sl)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        run_step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    loss = float(tr.loss.item())

    # ---- probe pass: eager steps with HIP events around the dominant kernels (same stream)
    probe = {}
    for i in range(args.probe_steps):
        load(i)
        tr.step(sb, sl, probe=probe)
    torch.cuda.synchronize()

    def avg_ms(name):
        ev = probe.get(name, [])
        return sum(s.elapsed_time(e) for s, e in ev) / max(1, len(ev))

    adam_ms, gather_ms = avg_ms("adam_table"), avg_ms("fields_fwd")
    # touched rows of one batch (for the table-Adam byte count): unique non-zero ids routed here
    b0 = batches[0][0]
    ids = torch.cat([b0["item_id"], b0["item_seq"].flatten()])
    ids = ids[(ids > 0) & (ids >= tr.rows_lo) & (ids < tr.rows_lo + tr.rows_local)]
    touched = int(torch.unique(ids).numel())
    if world > 1:
        tt = torch.tensor([touched], device=dev)
        dist.all_reduce(tt)
        touched = int(tt.item()) // world
    a_bytes = adam_table_bytes(tr.rows_local, d, touched)
    a_gbs = a_bytes / (adam_ms * 1e-3) / 1e9
    g_bytes = gather_bytes_per_sample(d) * B
    g_gbs = g_bytes / (gather_ms * 1e-3) / 1e9

    if rank == 0:
        samples = K * B * world
        out = {
            "metric": "training samples/sec (FiBiNET d=128, MicroLens-shaped synthetic, full train step)",
            "value": round(samples / dt, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(dt / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if args.dtype == "bf16" else "fp32",
            "data": "synthetic (MicroLens-shaped, seeded, HBM-resident; random-init weights)",
            "config": {"workload": "C3: FiBiNET emb_dim=128 + item_emb_d128, batch 8192/GPU, history 20, "
                                   "bf16 GEMM operands / fp32 accumulation + fp32 master weights and Adam",
                       "model": "MM_FiBiNET", "global_batch": B * world, "seq_len": L,
                       "item_rows": V, "item_rows_per_gpu": tr.rows_local, "emb_dim": d,
                       "parallelism": f"row-shard{world}" if world > 1 else "single",
                       "hipgraph": bool(graphs)},
            "roofline": {"kernel": "adam_table (dense Adam over the item-table shard)", "bound": "hbm",
                         "achieved": round(a_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(a_gbs / HBM_PEAK_GBS, 4), "traffic": None,
                         "bytes_per_launch": a_bytes, "avg_launch_ms": round(adam_ms, 4)},
            "roofline_gather": {"kernel": "fields_fwd (fused gather + LN + SENET)", "bound": "hbm",
                                "achieved": round(g_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": round(g_gbs / HBM_PEAK_GBS, 4), "bytes_per_launch": g_bytes,
                                "avg_launch_ms": round(gather_ms, 4)},
            "final_loss": round(loss, 5),
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args, world)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
