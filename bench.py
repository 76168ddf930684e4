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
  roofline:      the dominant kernel of the step (largest average launch time among the probed
                 ones), HIP events around its launches inside an eager probe pass (same stream),
                 algorithmic work per launch (bytes or FLOPs) / that time, against the HBM or
                 MFMA peak; traffic = PMC-measured HBM bytes per launch when committed;
  rooflines:     the same for every probed kernel (gather, lazy table-Adam catch-up, MLP GEMM);
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
MFMA_PEAK_TFS = 2500.0         # dense bf16 MFMA (2.5 PFLOP/s, no sparsity)
FP32_MFMA_PEAK_TFS = 157.0     # fp32 matrix
ROWS_PER_GPU = 1_250_000


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    # the lazy table Adam's per-row lag settles after ~1/p = V/touched-per-step steps: warm up
    # into steady-state training (warm-up steps are < 1 ms each)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--batch", type=int, default=8192, help="per-GPU batch")
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--rows-per-gpu", type=int, default=ROWS_PER_GPU)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=20)
    ap.add_argument("--probe-steps", type=int, default=10)
    return ap.parse_args()


def gather_bytes_per_sample(d: int, L: int = 20) -> int:
    # (L+1) rows requested + 23 int64 ids + 4 output rows (item, hist, likes, views)
    return (L + 1) * d * 4 + (L + 3) * 8 + 4 * d * 4


def catchup_bytes(rows: int, d: int, entries: int) -> int:
    # every row brought up to date: read + write p, m, v (24 B/elem) and last[] (8 B); the
    # claim list (4 B per entry)
    return rows * (24 * d + 8) + 4 * entries


def _pmc_traffic() -> dict:
    """HBM bytes per launch from the committed rocprofv3 PMC pass (profiles/*pmc*.json), if any."""
    import glob
    out = {}
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic*.json"))):
        try:
            out.update({k: v.get("bytes_per_launch") for k, v in json.load(open(f)).items()})
        except (OSError, ValueError, AttributeError):
            pass
    return out


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
    # rehearsal of the N > 1 path on a one-GPU box: FBN_BENCH_BACKEND=gloo puts every rank on
    # cuda:0 with host-staged collectives (RCCL refuses two ranks on one device); timings from
    # it are not scaling numbers
    backend = os.environ.get("FBN_BENCH_BACKEND", "nccl")
    rehearsal = backend != "nccl"
    if rehearsal:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    group = None
    if world > 1:
        if rehearsal:
            dist.init_process_group(backend)
        else:
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
                        init_state=init, stage_on_cpu=rehearsal)
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
        tt = torch.tensor([dt], device="cpu" if rehearsal else dev, dtype=torch.float64)
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

    # per-launch algorithmic work of the probed kernels (DESIGN.md "Measurement")
    b0 = batches[0][0]
    ids = torch.cat([b0["item_id"], b0["item_seq"].flatten()])
    ids = ids[(ids > 0) & (ids >= tr.rows_lo) & (ids < tr.rows_lo + tr.rows_local)]
    touched = int(torch.unique(ids).numel())
    if world > 1:
        tt = torch.tensor([touched], device="cpu" if rehearsal else dev)
        dist.all_reduce(tt)
        touched = int(tt.item()) // world
    window = -(-tr.rows_local // tr.lazy_window)
    rooflines = []

    def add(name, kernel, ms, work, unit, peak, bound, detail):
        if ms > 0:
            ach = work / (ms * 1e-3) / (1e9 if unit == "GB/s" else 1e12)
            rooflines.append({"kernel": kernel, "bound": bound, "achieved": round(ach, 1), "peak": peak, "unit": unit,
                              "frac": round(ach / peak, 4), "traffic": traffic.get(name), "avg_launch_ms": round(ms, 4),
                              "work_per_launch": work, "work_basis": detail})

    traffic = _pmc_traffic()
    add("fields_fwd", "fields_fwd (fused gather + history mean + LN + SENET)", avg_ms("fields_fwd"),
        gather_bytes_per_sample(d) * B, "GB/s", HBM_PEAK_GBS, "hbm", "SURVEY 8(d) 12,984 B/sample x batch")
    # the probed launch is the claimed-row pass only (the rolling window runs on the side stream);
    # with deferred table gradients it also reads each row's pending gradient vector (4 B x d) and
    # its pend entry (+8 B)
    dfr = getattr(tr, "deferred", False)
    add("adam_catchup", "adam_catchup (lazy table Adam: rows claimed this step)", avg_ms("adam_catchup"),
        catchup_bytes(touched, d, B * (L + 1)) + (touched * (4 * d + 8) if dfr else 0), "GB/s", HBM_PEAK_GBS, "hbm",
        f"touched {touched} rows x (24 B x d + 8 B{' + 4 B x d + 8 B deferred gradient' if dfr else ''}) "
        f"+ 4 B per entry")
    add("adam_window", "adam_catchup (lazy table Adam: rolling window, side stream)", avg_ms("adam_window"),
        catchup_bytes(window, d, 0), "GB/s", HBM_PEAK_GBS, "hbm",
        f"window {window} rows x (24 B x d + 8 B); VALU-bound replay of up to F steps per row")
    add("gemm_mlp0", "gemm MLP layer 1 (B x 15d -> 512, bf16 MFMA)", avg_ms("gemm_mlp0"),
        2.0 * B * 512 * 15 * d, "TFLOP/s", MFMA_PEAK_TFS if args.dtype == "bf16" else FP32_MFMA_PEAK_TFS, "mfma",
        "2 x B x 512 x 15d")
    if tr.table_adam == "eager":
        add("adam_table", "adam_table (eager: every untouched row each step)", avg_ms("adam_table"),
            24 * tr.rows_local * d + 4 * tr.rows_local, "GB/s", HBM_PEAK_GBS, "hbm", "24 B x rows x d + 4 B x rows")
    # the dominant kernel of the step's critical path (main stream; the window replay overlaps it)
    main_k = [r for r in rooflines if "side stream" not in r["kernel"]]
    dominant = max(main_k, key=lambda r: r["avg_launch_ms"]) if main_k else None

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
                       "hipgraph": bool(graphs), **({"rehearsal": backend} if rehearsal else {})},
            "roofline": dominant,
            "rooflines": rooflines,
            "table_adam": tr.table_adam,
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
