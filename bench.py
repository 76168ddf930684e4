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
                 ones), its launches timed by their own start / end events inside an eager probe
                 pass (the library launches every kernel with hipExtLaunchKernelGGL; armed per call
                 by _lib.KernelProbe: the kernel span rocprofv3 reports, no marker packets around it),
                 algorithmic work per launch (bytes or FLOPs) / that time, against the HBM or
                 MFMA peak; traffic = PMC-measured HBM bytes per launch when committed;
  rooflines:     the same for every probed kernel (gather, lazy table-Adam catch-up, MLP GEMM),
                 plus the gather and the layer-1 GEMM "alone" (eval-mode forwards with nothing on
                 the side stream: the in-step launches share the GPU with the table-Adam side work,
                 which is why a rocprof per-name average -- graph replays + probes + these -- sits
                 between the two; tools/step_launches.py lists one step's launches);
  host_enqueue_ms_per_step: host time to issue the K timed steps (graph replays or eager launches);
  host_wait_ms_per_step (N > 1 / the sharded one-rank job): of that, the host's wait for the routed-ahead
                 batch's overflow flag before each step -- back-pressure: the flag is ready ~1/3 into the
                 step before, so the host waits while the GPU still has ~2/3 of a step queued;
                 host_busy_ms_per_step = enqueue - wait (what the host needs per step);
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
LIVE_EVERY = 8       # one step program in 8 carries the recorded kernel-span probes (bench rooflines)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    # untimed warm-up steps; bench tops them up to 2F steps of priming (steady-state lazy Adam)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=8192, help="per-GPU batch")
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--rows-per-gpu", type=int, default=ROWS_PER_GPU)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "bf16_fwd", "fp32"],
                    help="bf16: every GEMM operand bf16; bf16_fwd: forward GEMM operands bf16, backward fp32; fp32")
    ap.add_argument("--no-graph", action="store_true", help="N = 1: no hipGraph capture (auto picks program / eager)")
    ap.add_argument("--mode", default="auto", choices=["auto", "program", "graph", "eager"],
                    help="N = 1: replay one recorded step program per batch (the native step driver, "
                         "csrc/plan.cpp), replay one hipGraph per batch, launch eagerly from Python, or (auto) "
                         "time all three for a few steps after priming and run the timed steps in the fastest")
    ap.add_argument("--main-priority", action="store_true",
                    help="run the step on a high-priority stream (the side stream stays at normal priority)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=20)
    ap.add_argument("--no-cpu-plan", dest="cpu_plan", action="store_false",
                    help="skip BASELINE.md 2's CPU-baseline plan (C1 / C2 shapes, 20 warm-up + 200 timed steps)")
    ap.add_argument("--cpu-plan-steps", type=int, default=200)
    ap.add_argument("--no-inference", dest="inference", action="store_false",
                    help="skip the inference leg (eval-mode drop-in forwards at batch 8192, src/Prediction.py:95-113)")
    ap.add_argument("--infer-batches", type=int, default=96)
    ap.add_argument("--probe-steps", type=int, default=10)
    ap.add_argument("--no-live-probes", dest="live_probes", action="store_false",
                    help="step programs without the kernel-span probes recorded into them (the in-step "
                         "rooflines then come from the eager probe pass)")
    ap.add_argument("--batches", type=int, default=0, help="distinct HBM-resident batches (default F + 32)")
    ap.add_argument("--lazy-window", type=int, default=0,
                    help="lazy table-Adam window F (rows per step: V/F; default: the trainer's, 128 at d >= 128, else 32)")
    ap.add_argument("--zipf", type=float, default=0.0,
                    help="item / history ids ~ Zipf(s) (SURVEY 8(d): 1.05) instead of uniform")
    ap.add_argument("--table-adam", default="lazy", choices=["lazy", "eager", "sparse"],
                    help="item-table Adam: lazy (exact replay, default), eager (every row each step), sparse "
                         "(opt-in non-parity C5 variant: touched rows only)")
    ap.add_argument("--no-prefetch", dest="prefetch", action="store_false",
                    help="N = 1: no ahead-of-time catch-up of the next batch's rows (fbn_adam_prefetch)")
    ap.add_argument("--prime", type=int, default=-1,
                    help="untimed priming steps before the warm-up (default: top the warm-up up to 2F)")
    ap.add_argument("--bn", default="local", choices=["local", "sync"],
                    help="N > 1 BatchNorm statistics: 'local' = per GPU, what the reference script does on a "
                         "multi-GPU box (nn.DataParallel, train_fibinet.py:69-70); 'sync' = over the global "
                         "batch (parity with one process on the global batch; 4 all-reduces per step)")
    ap.add_argument("--no-other-bn", action="store_true",
                    help="N > 1: skip the second measurement in the other BatchNorm mode")
    ap.add_argument("--no-fp32", dest="also_fp32", action="store_false",
                    help="skip the fp32 and bf16_fwd C3 measurements embedded in the line")
    return ap.parse_args()


def gather_bytes_per_sample(d: int, L: int = 20) -> int:
    # (L+1) rows requested + 23 int64 ids + 4 output rows (item, hist, likes, views)
    return (L + 1) * d * 4 + (L + 3) * 8 + 4 * d * 4


def catchup_bytes(rows: int, d: int, entries: int) -> int:
    # every row brought up to date: read + write p, m, v (24 B/elem) and last[] (8 B); the
    # claim list (4 B per entry)
    return rows * (24 * d + 8) + 4 * entries


def _pmc_traffic(dtype: str = "bf16") -> dict:
    """HBM bytes per launch from the newest committed rocprofv3 PMC pass (profiles/*pmc_traffic*.json)
    of this dtype's bench command (files named *_fp32_* hold the fp32 run's)."""
    import glob
    out = {}
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic*.json")))
    files = [f for f in files if ("fp32" in os.path.basename(f)) == (dtype == "fp32")]
    for f in files:
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


def cpu_baseline_plan(args):
    """BASELINE.md 2 / SURVEY 8(d)'s CPU-baseline plan: the oracle's train step (torch CPU restatement of
    src/train_fibinet.py:113-123) at the C1 shape (d 16, batch 256, the reference's 91 718-row vocab) and
    the C2 shape (d 16, batch 4096, 1 M rows), 20 warm-up + 200 timed steps each, on this host's cores."""
    from ctr_recommendation_amd.data import make_batch
    from oracle.fibinet_oracle import OracleTrainer, build_model
    threads = torch.get_num_threads()
    out = []
    for name, d, B, V in (("C1", 16, 256, 91_718), ("C2", 16, 4096, 1_000_000)):
        torch.manual_seed(2025)
        tr = OracleTrainer(build_model(None, {"embedding_dim": d, "vocab_size": V}), lr=1e-3, weight_decay=1e-5,
                           total_steps=1000)
        batches = [make_batch(7 + i, B, V) for i in range(4)]
        for i in range(20):
            tr.step(*batches[i % 4])
        n = args.cpu_plan_steps
        t0 = time.perf_counter()
        for i in range(n):
            tr.step(*batches[i % 4])
        dt = time.perf_counter() - t0
        out.append({"config": name, "value": round(n * B / dt, 1), "unit": "samples/s",
                    "ms_per_step": round(dt / n * 1e3, 3), "cores": threads, "kind": "port",
                    "sample": f"20 warm-up + {n} timed oracle train steps, d={d}, batch {B}, {V} item rows (fp32)"})
        del tr, batches
    return out


def _mean_ms(pairs) -> float:
    """Mean kernel span (ms) of a probe list: _lib.KernelProbe entries (the library's kernels, timed by
    their own start / end events: what rocprofv3 reports) or torch event pairs; probes whose call
    launched nothing are skipped."""
    vals = [a.elapsed_time(e) for a, e in pairs]
    vals = [v for v in vals if v >= 0]
    return sum(vals) / len(vals) if vals else 0.0


def inference_leg(args, dev, dtype):
    """Inference throughput (SURVEY 6's other derived figure, src/Prediction.py:95-113): the drop-in
    MM_FiBiNET in eval mode, batch 8192, d = 128, `model(batch_dict)` then `y_pred.cpu()` per batch --
    the reference loop (ctr_recommendation_amd.predict.predict) over HBM-resident synthetic batches, so
    the host collate (pandas, 4 workers) is out of the timed region.  Also the gather's roofline inside
    those forwards (HIP events around fields_fwd, same stream)."""
    from ctr_recommendation_amd import ops
    from ctr_recommendation_amd.data import make_device_batches
    from ctr_recommendation_amd.model_fibinet import build_model
    from ctr_recommendation_amd.predict import predict
    d, B, V, L = args.dim, args.batch, args.rows_per_gpu, 20
    torch.manual_seed(2025)
    model = build_model(None, {"embedding_dim": d, "vocab_size": 4, "compute_dtype": dtype})
    g = torch.Generator(device=dev)
    g.manual_seed(2025)
    table = torch.randn((V, d), generator=g, device=dev)
    table[0].zero_()
    model.item_emb.weight = torch.nn.Parameter(table)
    model.to(dev).eval()
    nb = 32
    xs = [b for b, _ in make_device_batches(nb, B, V, L, dev, seed=4242)]
    predict(model, xs[:4])                              # warm-up
    torch.cuda.synchronize()
    n = max(nb, args.infer_batches)
    t0 = time.perf_counter()
    preds = predict(model, [xs[i % nb] for i in range(n)])
    dt = time.perf_counter() - t0
    assert preds.shape == (n * B,)
    # the gather inside the same eval-mode forwards, timed by events on its stream
    p = {k: t for k, t in model.named_parameters()}
    p.update(model._buffers_dict())
    cfg = model._fwd_cfg()
    cfg.L = L
    probe = {}
    with torch.no_grad():
        for j in range(12):
            torch.cuda._sleep(2_000_000)
            ops.forward(p, xs[j % nb], cfg, None, probe=probe)
    torch.cuda.synchronize()
    ms = _mean_ms(probe["fields_fwd"][2:])
    work = gather_bytes_per_sample(d) * B
    ach = work / (ms * 1e-3) / 1e9
    out = {"value": round(n * B / dt, 1), "unit": "samples/s", "ms_per_batch": round(dt / n * 1e3, 4),
           "batches": n, "batch": B, "dtype": dtype, "emb_dim": d, "item_rows": V,
           "loop": "src/Prediction.py:106-113 (model(batch_dict); y_pred.cpu().numpy() per batch) through the drop-in "
                   "MM_FiBiNET, eval mode; batches HBM-resident (no host collate)",
           "roofline": {"kernel": "fields_fwd (eval-mode forward)", "bound": "hbm", "achieved": round(ach, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                        "traffic": None, "avg_launch_ms": round(ms, 4), "work_per_launch": work,
                        "work_basis": "SURVEY 8(d) 12,984 B/sample x batch"}}
    del model, xs, table
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def _initial_state(cfg, V, world, rank, dev):
    """Seeded init: small params from build_model; the N(0,1) table (row 0 = padding = 0) built on the
    device -- each rank only materialises its own shard (the trainer slices init[...][lo:hi])."""
    torch.manual_seed(2025)
    from ctr_recommendation_amd.model_fibinet import build_model
    init = dict(build_model(None, dict(cfg, vocab_size=4)).state_dict())
    g = torch.Generator(device=dev)
    g.manual_seed(2025)
    d = cfg["embedding_dim"]
    if world == 1:
        table = torch.randn((V, d), generator=g, device=dev)
        table[0].zero_()
        init["item_emb.weight"] = table
        return init

    class _Shard:
        shape = (V, d)

        def __getitem__(self, sl):
            n = min(V, sl.stop) - sl.start
            t = torch.randn((n, d), generator=g, device=dev)
            if sl.start == 0:
                t[0].zero_()
            return t
    init["item_emb.weight"] = _Shard()
    return init


# FBN_BENCH_SHARD=1 (under torch.distributed.run, one rank): the row-sharded N > 1 step at N = 1
# over RCCL -- the per-GPU cost of the sharded path without any peer (scaling diagnostics)
FORCE_SHARD = os.environ.get("FBN_BENCH_SHARD") == "1"


AB_CYCLES = 3      # native_ab: passes over its batches after the recording pass


def _ab_agree(ok: bool, first_diff: int, dev) -> tuple:
    """Every rank's verdict of the lockstep A/B -> the job's: valid only if valid on EVERY rank; the
    first step that differed anywhere (-1: none).  One MIN all-reduce on the default group."""
    t = torch.tensor([1 if ok else 0, first_diff if first_diff >= 0 else 1 << 30], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    fd = int(t[1])
    return bool(t[0]), (-1 if fd >= 1 << 30 else fd)


def native_ab(args, world, rank, dev):
    """N > 1 (and the one-rank sharded job): validate the fast collective path before timing it.

    The sharded step runs two ways from the same seeded state over the same batches, both in
    deterministic mode (the fixed-point owner fold: no order-dependent reduction left in the step):
      A  native RCCL on the step's stream (csrc/comm.cpp) + the fixed-capacity exchange recorded as
         step programs -- the fast path, never run above one rank before this job;
      B  torch.distributed's collectives, eager steps (the compute between exchanges as hipGraph
         segments) -- the conservative path.
    A runs first, through the exchange's calibration steps, the recording pass and AB_CYCLES replay
    passes, under the native communicators' watchdog (FBN_AB_TIMEOUT_S, default 120 s: a rank whose
    peer never posts aborts instead of hanging); its health is agreed over every rank; then B runs the
    same steps.  Valid iff every step's loss and, after the flush, the table, its Adam moments and the
    dense parameters and moments are bitwise equal on every rank.  Returns the verdict (and the first
    differing step) for the headline's choice of path."""
    from ctr_recommendation_amd import _lib
    from ctr_recommendation_amd.data import make_device_batches
    from ctr_recommendation_amd.exchange import NativeComm
    from ctr_recommendation_amd.trainer import FC_CALIB_STEPS, FiBiNETTrainer
    t_start = time.perf_counter()
    d, B, L = args.dim, args.batch, 20
    V = args.rows_per_gpu * world
    cfg = {"embedding_dim": d, "vocab_size": V, "compute_dtype": args.dtype}
    nb = 4
    batches = make_device_batches(nb + FC_CALIB_STEPS, B, V, L, dev, seed=9090 + rank, zipf=args.zipf)
    order = [nb + k for k in range(FC_CALIB_STEPS)] + [nb - 1] + list(range(nb)) * (1 + AB_CYCLES)
    total = len(order) + 4
    names = ("E", "Em", "Ev", "flat_p", "flat_m", "flat_v")

    def run(native: bool):
        init = _initial_state(cfg, V, world, rank, dev)
        tr = FiBiNETTrainer(cfg, total_steps=total, batch_size=B, device=dev, rank=rank, world=world, init_state=init,
                            shard=True, deterministic=True, sync_bn=args.bn == "sync", native_comm=native)
        del init
        if native:
            assert tr.native_comm is not None
            _lib.call("fbn_comm_watch", int(float(os.environ.get("FBN_AB_TIMEOUT_S", "120")) * 1000))
        losses, progs, pool = [], {}, torch.cuda.MemPool() if native else None
        for i, j in enumerate(order):
            b, y = batches[j]
            nxt = batches[order[i + 1]][0] if i + 1 < len(order) else batches[order[0]][0]
            if native and i > FC_CALIB_STEPS:
                if j not in progs:
                    progs[j] = tr.record_program(b, y, next_batch=nxt, pool=pool)
                else:
                    tr.run_program(progs[j])
            else:
                tr.step(b, y, next_batch=nxt)
            losses.append(tr.loss.clone())
        tr.flush()
        torch.cuda.synchronize()
        tr.check_ids()
        info = {"fc_active": bool(tr.xchg.fc_active), "fallbacks": tr.xchg.fc_fallbacks,
                "programs": len(progs), "collectives": "native" if tr.native_comm is not None else "torch"}
        state = {n: getattr(tr, n) for n in names}
        return tr, torch.stack(losses), state, info

    ok_a, err = True, None
    tra = la = sa = ia = None
    try:
        tra, la, sa, ia = run(True)
        ok_a = ia["fc_active"] and ia["programs"] == nb
        if not ok_a:
            err = f"native path did not run as step programs over the fixed-capacity exchange: {ia}"
    except Exception as e:           # a watchdog abort, an RCCL error, a recording refused on this rank
        ok_a, err = False, f"{type(e).__name__}: {e}"[:400]
    if not ok_a:
        print(f"[bench] rank {rank}: native path failed the A/B: {err}", file=sys.stderr, flush=True)
    healthy, _ = _ab_agree(ok_a, -1, dev)
    out = {"steps": len(order), "batches": nb, "deterministic": True, "native_healthy": healthy,
           "watchdog_fired": NativeComm.watchdog_fired()}
    if not healthy:
        if tra is not None:
            tra.close()
        out.update(validated=False, use_native=False, first_diff_step=-1,
                   reason=err or "another rank's native path failed", seconds=round(time.perf_counter() - t_start, 1))
        return out
    try:
        trb, lb, sb, ib = run(False)
        torch_err = None
    except Exception as e:           # the torch.distributed path itself failed on this rank
        trb, torch_err = None, f"{type(e).__name__}: {e}"[:400]
    torch_ok, _ = _ab_agree(torch_err is None, -1, dev)
    if not torch_ok:
        # the conservative path is the broken one: the native path ran healthy on every rank, so it
        # is timed -- unvalidated, and the line says so
        for t in (tra, trb):
            if t is not None:
                t.close()
        out.update(validated=False, use_native=True, first_diff_step=-1, native=ia,
                   reason=f"the torch.distributed path failed: {torch_err or 'on another rank'}",
                   seconds=round(time.perf_counter() - t_start, 1))
        return out
    diff = (la != lb).nonzero()
    first = int(diff[0, 0]) if diff.numel() else -1
    same = {n: bool(torch.equal(sa[n], sb[n])) for n in names}
    ok = first < 0 and all(same.values())
    valid, first_all = _ab_agree(ok, first, dev)
    for t in (tra, trb):
        t.close()
    del tra, trb, sa, sb
    out.update(validated=valid, use_native=valid, first_diff_step=first_all, equal_this_rank=same, native=ia,
               torch=ib, loss_last=(float(la[-1]), float(lb[-1])), seconds=round(time.perf_counter() - t_start, 1))
    if not valid:
        out["reason"] = ("losses first differ at step %d" % first_all) if first_all >= 0 else "final state differs"
    return out


def measure(args, dtype, world, rank, dev, rehearsal, backend, bn=None, native=None):
    """Build a trainer for `dtype`, bring it to steady state, time K steps; returns the result dict.
    native (N > 1): True / False = native RCCL + step programs / torch.distributed (None: FBN_NATIVE_COMM)."""
    from ctr_recommendation_amd.data import make_device_batches
    from ctr_recommendation_amd import ops
    from ctr_recommendation_amd.trainer import FiBiNETTrainer
    from ctr_recommendation_amd import trainer as trmod

    d, B, L = args.dim, args.batch, 20
    V = args.rows_per_gpu * world
    cfg = {"embedding_dim": d, "vocab_size": V, "compute_dtype": dtype}
    K, W = args.steps, args.warmup
    from ctr_recommendation_amd.trainer import default_lazy_window
    F = args.lazy_window or default_lazy_window(d)   # lazy table-Adam window (the trainer's default)
    # fresh ids every step: more distinct HBM-resident batches than the window F, so every row a
    # timed step claims was last touched at the lag fresh uniform ids give (bounded by F), never
    # replayed from a batch seen a few steps earlier
    nb = args.batches if args.batches else F + 32
    # steady state of the lazy table Adam whatever --warmup says: a row's replay length settles
    # only after ~2F steps; warm-up steps are < 1 ms each
    prime = max(0, 2 * F - W) if args.prime < 0 else args.prime
    sharded = world > 1 or FORCE_SHARD
    use_graph = not sharded and not args.no_graph and args.mode in ("auto", "graph")
    # step programs: the single-GPU step, and the sharded step in the fixed-capacity exchange form over
    # RCCL on the step's stream (the one-rank job; N > 1 with FBN_NATIVE_COMM=1)
    from ctr_recommendation_amd.exchange import native_comm_wanted
    shard_prog = sharded and trmod._FC and native_comm_wanted(dev, None, rehearsal, force=native)
    use_prog = (not sharded or shard_prog) and args.mode in ("auto", "program") and args.table_adam == "lazy"
    if use_prog:
        prime = max(prime, nb)            # every batch's program is recorded (a real step each) while priming
    modes = [m for m, ok in (("program", use_prog), ("graph", use_graph), ("eager", True)) if ok]
    trial_n = 16 if (args.mode == "auto" and len(modes) > 1) else 0
    total = 2 + trmod.FC_CALIB_STEPS + (nb if use_graph else 0) + prime + W + K + args.probe_steps + 16 + 2 * len(modes) * trial_n
    if args.main_priority:
        # the step's own stream at high priority: the hardware queue arbiter then dispatches its
        # workgroups ahead of the table-Adam side stream's when both have work pending
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=-1))
    init = _initial_state(cfg, V, world, rank, dev)
    tr = FiBiNETTrainer(cfg, total_steps=total, batch_size=B, device=dev, rank=rank, world=world,
                        init_state=init, stage_on_cpu=rehearsal, lazy_window=F, prefetch_rows=args.prefetch,
                        table_adam=args.table_adam,
                        shard=sharded, sync_bn=(bn or args.bn) == "sync", native_comm=native)
    del init
    batches = make_device_batches(nb, B, V, L, dev, seed=2025 + rank, zipf=args.zipf)
    graphs = []
    if use_graph:
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            tr.step(*batches[0])                  # side-stream warm-up required before capture
        torch.cuda.current_stream().wait_stream(s)
        # one graph per HBM-resident batch (shared memory pool): every step is one replay
        pool = None
        for j, (b, y) in enumerate(batches):
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, pool=pool):
                tr.step(b, y, next_batch=batches[(j + 1) % nb][0])   # next batch's rows caught up ahead
            pool = gr.pool()
            graphs.append(gr)
        torch.cuda.synchronize()

    mode_now = [modes[0]]
    progs = [None] * nb
    # kernel-span probes recorded into every program: each replay re-arms them, so right after the timed
    # steps the programs replayed there hold the spans of THOSE launches (rooflines of the timed region)
    # (one program in LIVE_EVERY carries them: a probed kernel launch costs ~2 us, so probing every
    # step would slow the very steps it times)
    live = [({} if j % LIVE_EVERY == 0 else None) for j in range(nb)] if (use_prog and args.live_probes) else None
    prog_pool = torch.cuda.MemPool() if use_prog else None     # one private pool for every program

    def run_step(i):
        j = i % nb
        if mode_now[0] == "graph":
            graphs[j].replay()
        elif mode_now[0] == "program" and progs[j] is not None:
            tr.run_program(progs[j])
        elif mode_now[0] == "program":
            # first visit of this batch: a real step, recorded (the program replays it from now on)
            b, y = batches[j]
            progs[j] = tr.record_program(b, y, next_batch=batches[(i + 1) % nb][0], pool=prog_pool,
                                         probe=live[j] if live else None)   # None: unprobed program
        else:
            # the HBM-resident batch itself: N > 1 routes the next batch during this step (no
            # mid-step host sync); N = 1 catches its rows up ahead and pre-claims them
            b, y = batches[j]
            tr.step(b, y, next_batch=batches[(i + 1) % nb][0])

    if use_prog and sharded:
        # the exchange's calibration steps (host split sizes), after which it is fixed-capacity
        for k in range(trmod.FC_CALIB_STEPS):
            tr.step(batches[nb - 2 - k][0], batches[nb - 2 - k][1], next_batch=batches[nb - 1 - k][0])
    if use_prog:
        # the step before the first recording prefetches (and pre-claims) batch 0, as the step before
        # every replay of its program will (the last batch's program); sharded: routes it ahead
        tr.step(batches[-1][0], batches[-1][1], next_batch=batches[0][0])
    i = 0
    for j in range(prime + W):
        run_step(i)
        i += 1
        if (j + 1) % 64 == 0 and rank == 0:
            print(f"[bench] {dtype}: {j + 1}/{prime + W} untimed steps", file=sys.stderr, flush=True)
    # auto: a timed trial of both launch modes at steady state (graph replays and eager steps share
    # every persistent buffer -- table, moments, deferred-gradient ring, pre-claims -- so the modes
    # interleave freely: tests/test_gpu_trainer.py::test_graph_eager_interleave_bit_identical)
    trial = {}
    if trial_n:
        for rnd in range(2):
            for mode in modes:
                mode_now[0] = mode
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(trial_n):
                    run_step(i)
                    i += 1
                torch.cuda.synchronize()
                trial.setdefault(mode, []).append((time.perf_counter() - t0) / trial_n * 1e3)
        mode_now[0] = min(modes, key=lambda m: min(trial[m]))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if tr.xchg is not None:
        tr.xchg.host_wait_s = 0.0
    t0 = time.perf_counter()
    i_timed = i
    for _ in range(K):
        run_step(i)
        i += 1
    t_host = time.perf_counter() - t0            # host enqueue time of the K steps
    t_wait = tr.xchg.host_wait_s if tr.xchg is not None else 0.0   # of which waiting for the routed-ahead batch
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], device="cpu" if rehearsal else dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    tr.check_ids()                                # ids in range, no step past total_steps
    loss = float(tr.loss.item())

    # ---- replay length of the claimed rows at this point of steady state (mean steps per row)
    b_next = batches[i % nb][0]
    ids = torch.cat([b_next["item_id"], b_next["item_seq"].flatten()])
    ids = ids[(ids > 0) & (ids >= tr.rows_lo) & (ids < tr.rows_lo + tr.rows_local)]
    uniq = torch.unique(ids) - tr.rows_lo
    lag = (tr.step_dev.to(torch.int64) - tr.last[uniq].to(torch.int64)).double().mean().item()
    # rows the next step's claimed-row catch-up still has to replay (with the next-batch prefetch,
    # only rows the previous batch also touched; the rest were replayed beside the previous step)
    stale = int((tr.last[uniq] < tr.step_dev).sum().item())
    prefetch = bool(getattr(tr, "prefetch_rows", False)) and world == 1
    # N > 1 (and the one-rank sharded run): the owner catches the next step's requested rows up
    # ahead (fbn_adam_prefetch_rows), so the claimed-row catch-up replays only the stale ones too
    owner_pf = bool(getattr(tr, "prefetch_owner", False)) and tr.xchg is not None

    # ---- probe pass: eager steps with the dominant kernels' spans probed (_lib.KernelProbe)
    probe = {}
    for _ in range(args.probe_steps):
        b, y = batches[i % nb]
        i += 1
        # a ~10 ms spin ahead of the step keeps the GPU behind the host's launches, so the step's
        # kernels run back to back as in the timed replays, not at the host's pace; the
        # HBM-resident batches themselves are passed (as in the graphs), so the next-batch
        # prefetch's claims are taken up exactly as in the timed replays
        torch.cuda._sleep(20_000_000)
        tr.step(b, y, probe=probe, next_batch=batches[i % nb][0] if world == 1 else None)
    torch.cuda.synchronize()
    # the same steps with the side-stream passes on the main stream: every kernel alone
    serial = {}
    if world == 1 and tr.xchg is None:
        side = tr.side
        tr.side = torch.cuda.current_stream(dev)
        for _ in range(max(4, args.probe_steps // 2)):
            b, y = batches[i % nb]
            i += 1
            torch.cuda._sleep(20_000_000)
            tr.step(b, y, probe=serial, next_batch=batches[i % nb][0])
        torch.cuda.synchronize()
        tr.side = side

    # the gather alone: eval-mode forwards of the same batches with nothing on the side stream (the
    # probe above times it inside the step, beside the table-Adam passes)
    iso = {}
    if world == 1:
        cfg_iso = ops.FwdConfig(**{**tr.fcfg.__dict__, "training": False})
        cfg_iso.L = L
        for j in range(12):
            torch.cuda._sleep(2_000_000)
            ops.forward(tr.p, batches[j % nb][0], cfg_iso, None, err=tr.err, probe=iso)
        torch.cuda.synchronize()

    # the in-step rooflines from the timed replays themselves (step programs with recorded probes): the
    # programs of the timed steps (each replayed once when K <= the number of batches) hold their spans
    timed_src = None
    if live and mode_now[0] == "program":
        timed_src = {}
        for jj in sorted({t % nb for t in range(i_timed, i_timed + K)}):
            for name, pairs in (live[jj] or {}).items():
                timed_src.setdefault(name, []).extend(pairs)
        for name, pairs in timed_src.items():
            probe[name] = pairs            # replaces the eager probe steps' in-step values

    def avg_ms(name, src=None):
        # the first two launches of an explicit source (the eval-mode forwards, the serialised probe
        # steps) carry first-iteration warm-up; the in-step probe follows the timed steps (warm)
        return _mean_ms((probe if src is None else src).get(name, [])[2 if src is not None else 0:])

    touched = int(uniq.numel())
    if world > 1:
        tt = torch.tensor([touched], device="cpu" if rehearsal else dev)
        dist.all_reduce(tt)
        touched = int(tt.item()) // world
    window = -(-tr.rows_local // tr.lazy_window)
    # the committed PMC passes are of the default C3 command: their bytes mean nothing for another
    # shape (C2, the C5 shard), so other workloads carry traffic null
    c3 = (d, B, args.rows_per_gpu, args.zipf) == (128, 8192, ROWS_PER_GPU, 0.0)
    traffic = _pmc_traffic(dtype) if c3 else {}
    rooflines = []

    def add(name, kernel, ms, work, unit, peak, bound, detail):
        if ms <= 0:
            return
        scale = 1e9 if unit == "GB/s" else 1e12
        ach = work / (ms * 1e-3) / scale
        r = {"kernel": kernel, "bound": bound, "achieved": round(ach, 1), "peak": peak, "unit": unit,
             "frac": round(ach / peak, 4), "traffic": traffic.get(name), "avg_launch_ms": round(ms, 4),
             "work_per_launch": work, "work_basis": detail}
        if unit == "GB/s" and traffic.get(name):
            # the same launch time against the PMC-measured HBM bytes (what actually moved)
            r["achieved_traffic"] = round(traffic[name] / (ms * 1e-3) / 1e9, 1)
            r["frac_traffic"] = round(r["achieved_traffic"] / peak, 4)
        rooflines.append(r)

    add("fields_fwd", "fields_fwd (fused gather + history mean + LN + SENET)", avg_ms("fields_fwd"),
        gather_bytes_per_sample(d) * B, "GB/s", HBM_PEAK_GBS, "hbm", "SURVEY 8(d) 12,984 B/sample x batch")
    if iso:
        add("fields_fwd", "fields_fwd alone (eval-mode forward, no side-stream work)", avg_ms("fields_fwd", iso),
            gather_bytes_per_sample(d) * B, "GB/s", HBM_PEAK_GBS, "hbm", "SURVEY 8(d) 12,984 B/sample x batch")
    dfr = getattr(tr, "deferred", False)
    # claimed-row catch-up: every entry's id, claim, slot and last (20 B) + the rows it replays
    crit = stale if (prefetch or owner_pf) else touched
    # the step head: the claims' launch also converts the bf16 operand images (fbn_adam_claim_catchup_conv):
    # Wa, Wa^T (512 x 15d), Wb, Wb^T (256 x 512), W, W^T (d x d), Wp (d x 128), x (B x 128); 4 B in, 2 B out
    head_conv = not sharded and dtype == "bf16" and trmod._HEAD_CONV and trmod._W16_MODE == "main"
    conv_bytes = 6 * (2 * 512 * 15 * d + 2 * 256 * 512 + 2 * d * d + d * 128 + B * 128) if head_conv else 0
    add("adam_catchup", "adam_catchup (lazy table Adam: rows claimed this step"
        + ("; the bf16 image conversion in the same launch)" if head_conv else ")"), avg_ms("adam_catchup"),
        catchup_bytes(crit, d, 5 * B * (L + 1)) + (crit * (4 * d + 8) if dfr else 0) + conv_bytes, "GB/s",
        HBM_PEAK_GBS, "hbm",
        f"{B * (L + 1)} entries x 20 B + {crit} replayed rows x (24 B x d + 8 B"
        f"{' + 4 B x d + 8 B deferred gradient' if dfr else ''}); mean lag {lag:.1f} steps over the {touched} rows"
        + (f" + {conv_bytes} B of bf16 images (6 B per element)" if head_conv else ""))
    if prefetch:
        ahead = max(0, touched - stale)
        pf_work = catchup_bytes(ahead, d, 5 * B * (L + 1)) + (ahead * (4 * d + 8) if dfr else 0)
        pf_basis = f"~{ahead} rows x (24 B x d + 8 B + deferred gradient) + {B * (L + 1)} entries x 20 B"
        add("adam_prefetch", "adam_prefetch (next batch's rows caught up ahead, side stream)", avg_ms("adam_prefetch"),
            pf_work, "GB/s", HBM_PEAK_GBS, "hbm", pf_basis)
        if serial:
            add("adam_prefetch", "adam_prefetch alone (serialised probe step, nothing beside it)",
                avg_ms("adam_prefetch", serial), pf_work, "GB/s", HBM_PEAK_GBS, "hbm", pf_basis)
    add("adam_window", "adam_catchup (lazy table Adam: rolling window, side stream)", avg_ms("adam_window"),
        catchup_bytes(window, d, 0), "GB/s", HBM_PEAK_GBS, "hbm",
        f"window {window} rows x (24 B x d + 8 B); VALU-bound replay of up to F steps per row")
    if serial:
        add("adam_window", "adam_catchup rolling window alone (serialised probe step)", avg_ms("adam_window", serial),
            catchup_bytes(window, d, 0), "GB/s", HBM_PEAK_GBS, "hbm",
            f"window {window} rows x (24 B x d + 8 B); VALU-bound replay of up to F steps per row")
    # the layer-1 forward GEMM takes bf16 operands in bf16 AND bf16_fwd mode (priced against the bf16
    # peak), fp32 operands (v_mfma_f32_32x32x2_f32) only in fp32 mode
    fwd_peak = FP32_MFMA_PEAK_TFS if dtype == "fp32" else MFMA_PEAK_TFS
    fwd_isa = "fp32 MFMA" if dtype == "fp32" else "bf16 MFMA"
    add("gemm_mlp0", f"gemm MLP layer 1 (B x 15d -> 512, {fwd_isa})", avg_ms("gemm_mlp0"),
        2.0 * B * 512 * 15 * d, "TFLOP/s", fwd_peak, "mfma", "2 x B x 512 x 15d")
    if iso:
        add("gemm_mlp0", f"gemm MLP layer 1 alone (eval-mode forward, no side-stream work, {fwd_isa})",
            avg_ms("gemm_mlp0", iso), 2.0 * B * 512 * 15 * d, "TFLOP/s", fwd_peak, "mfma", "2 x B x 512 x 15d")
    # the four weight-gradient GEMMs in their one grouped launch (bf16 mode): dWa, dWb, dW, dWp
    add("wgrad_group", "gemm weight gradients, grouped launch (dWa + dWb + dW + dWp, bf16 MFMA)",
        avg_ms("wgrad_group"), 2.0 * B * (512 * 15 * d + 256 * 512 + 5 * d * d + 128 * d), "TFLOP/s", MFMA_PEAK_TFS,
        "mfma", "2 x B x (512 x 15d + 256 x 512 + 5 d^2 + 128 d)")
    if tr.table_adam == "eager":
        add("adam_table", "adam_table (eager: every untouched row each step)", avg_ms("adam_table"),
            24 * tr.rows_local * d + 4 * tr.rows_local, "GB/s", HBM_PEAK_GBS, "hbm", "24 B x rows x d + 4 B x rows")
    main_k = [r for r in rooflines if "side stream" not in r["kernel"] and " alone " not in r["kernel"]]
    dominant = max(main_k, key=lambda r: r["avg_launch_ms"]) if main_k else None
    out = {"dt": dt, "t_host": t_host, "t_wait": t_wait, "K": K, "W": W, "B": B, "L": L, "V": V, "d": d, "rows_local": tr.rows_local, "loss": loss,
           "rooflines": rooflines, "roofline": dominant, "table_adam": tr.table_adam,
           "graphs": mode_now[0] == "graph", "launch_mode": mode_now[0],
           "probe_source": ("the timed step-program replays (kernel-span probes recorded into the programs)"
                            if timed_src else "eager probe steps after the timed region"),
           "collectives": (None if not sharded else "RCCL on the step's stream (csrc/comm.cpp)"
                           if tr.native_comm is not None else "torch.distributed process group"),
           "mode_trial_ms_per_step": {k: [round(x, 4) for x in v] for k, v in trial.items()} if trial else None,
           "prime": prime, "batches": nb, "lag": lag, "stale": stale, "touched": touched, "prefetch": prefetch}
    del graphs, progs, tr, batches
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def _workload(args, r) -> str:
    """config.workload: which BASELINE config this line measures, and in which precision."""
    prec = {"bf16": "every GEMM operand bf16 (forward and backward) / fp32 accumulation + fp32 master weights, "
                    "gradients and Adam",
            "bf16_fwd": "forward GEMM operands bf16 / fp32 accumulation, backward GEMMs and everything else fp32",
            "fp32": "fp32 throughout"}[args.dtype]
    d, B, rows = r["d"], r["B"], r["rows_local"]
    if d == 16 and B == 4096:
        name = f"C2: FiBiNET emb_dim=16, {rows} item rows, batch 4096/GPU, history 20 (item_emb_d128 input)"
    elif d == 128 and rows >= 10_000_000:
        name = (f"C5 per-GPU shard: FiBiNET emb_dim=128 + item_emb_d128, {rows} item rows on this GPU "
                f"(100 M / 8), batch {B}/GPU, history 20")
    elif d == 128:
        name = f"C3: FiBiNET emb_dim=128 + item_emb_d128, batch {B}/GPU, history 20"
    else:
        name = f"FiBiNET emb_dim={d}, batch {B}/GPU, {rows} item rows/GPU, history 20"
    return f"{name}, {prec}"



def _release() -> None:
    """The finished line's trainer and its cached blocks go back to the device."""
    import gc
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _child_line(dtype: str):
    """One embedded line measured in a process of its own (this bench, this dtype only, the parent's
    other arguments): a line measured in the process after another one ran ~4-5 % slower than on its
    own -- whichever ran third (c3_bf16_fwd 0.647-0.659 after the fp32 line vs 0.614-0.618 before it
    or alone; the fp32 line 1.16 vs 1.12), with or without releasing the allocator and with 15 s of
    idle between lines.  None if the child fails (the caller then measures in process)."""
    import subprocess
    argv, skip = [], False
    for x in sys.argv[1:]:
        if skip:
            skip = False
            continue
        if x == "--dtype":
            skip = True
            continue
        if not x.startswith("--dtype="):
            argv.append(x)
    cmd = [sys.executable, os.path.abspath(__file__)] + argv + [
        "--dtype", dtype, "--no-fp32", "--no-cpu-baseline", "--no-cpu-plan", "--no-inference"]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
        if r.returncode != 0 or not lines:
            print(f"[bench] {dtype} line in a child process failed (rc {r.returncode}): measuring in process",
                  file=sys.stderr, flush=True)
            return None
        d = json.loads(lines[-1])
        return {"K": d["steps"], "dt": d["ms_per_step"] * d["steps"] / 1e3, "roofline": d["roofline"],
                "loss": d["final_loss"], "process": "own"}
    except Exception as e:      # noqa: BLE001 -- an embedded line must not take the headline down
        print(f"[bench] {dtype} line in a child process failed ({e!r}): measuring in process", file=sys.stderr,
              flush=True)
        return None

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
    if world > 1 or FORCE_SHARD:
        if rehearsal:
            dist.init_process_group(backend)
        else:
            dist.init_process_group("nccl", device_id=dev)

    # N > 1 on RCCL: validate the native-RCCL + step-program path against torch.distributed's (lockstep
    # A/B, deterministic, bitwise) before timing it; the headline runs the validated path, the other
    # one is timed beside it.  FBN_BENCH_AB=0 skips the A/B (FBN_NATIVE_COMM then decides)
    ab, native, torch_line, native_err = None, None, None, None
    if (world > 1 or FORCE_SHARD) and not rehearsal and os.environ.get("FBN_BENCH_AB", "1") != "0":
        ab = native_ab(args, world, rank, dev)
        native = bool(ab["use_native"])
        _release()
        if rank == 0:
            print(f"[bench] native-RCCL A/B: {json.dumps(ab)}", file=sys.stderr, flush=True)
    if native:
        try:
            r = measure(args, args.dtype, world, rank, dev, rehearsal, backend, native=True)
            ok = True
        except Exception as e:       # a watchdog abort mid-run: every rank falls back together
            ok, native_err = False, f"{type(e).__name__}: {e}"[:400]
            print(f"[bench] rank {rank}: native headline failed: {native_err}", file=sys.stderr, flush=True)
        ok_all, _ = _ab_agree(ok, -1, dev)
        _release()
        if ok_all and ab.get("torch") is not None:      # (the torch path ran in the A/B)
            torch_line = measure(args, args.dtype, world, rank, dev, rehearsal, backend, native=False)
        else:
            native = False
            r = measure(args, args.dtype, world, rank, dev, rehearsal, backend, native=False)
    else:
        r = measure(args, args.dtype, world, rank, dev, rehearsal, backend,
                    native=None if ab is None else False)
    alt = alt16 = None
    if args.also_fp32 and args.dtype == "bf16" and world == 1:
        # each in a process of its own (_child_line), the headline's state released first
        _release()
        # the reference computes in fp32 throughout: the same C3 step with fp32 GEMM operands
        alt = _child_line("fp32") or measure(args, "fp32", world, rank, dev, rehearsal, backend)
        # C3's literal wording ("bf16 fwd / fp32 grad accum"): bf16 forward GEMMs, fp32 backward
        alt16 = _child_line("bf16_fwd") or measure(args, "bf16_fwd", world, rank, dev, rehearsal, backend)
    inf = None
    if world == 1 and args.inference and not FORCE_SHARD:
        inf = {m: inference_leg(args, dev, m) for m in ("fp32", "bf16")}
    other_bn = None
    if world > 1 and not args.no_other_bn:
        # both BatchNorm modes at N > 1: the other one as an embedded line (SyncBN = the parity mode)
        _release()
        other_bn = measure(args, args.dtype, world, rank, dev, rehearsal, backend,
                           bn="sync" if args.bn == "local" else "local", native=native)

    if rank == 0:
        K, B, dt = r["K"], r["B"], r["dt"]
        out = {
            "metric": f"training samples/sec (FiBiNET d={r['d']}, MicroLens-shaped synthetic, full train step)",
            "value": round(K * B * world / dt, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(dt / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": f"synthetic (MicroLens-shaped, seeded, HBM-resident, {r['batches']} distinct batches cycled: "
                    f"fresh ids every step, "
                    + (f"Zipf({args.zipf}) item / history ids" if args.zipf > 0 else "uniform ids")
                    + "; random-init weights)",
            "config": {"workload": _workload(args, r),
                       "model": "MM_FiBiNET", "global_batch": B * world, "seq_len": r["L"],
                       "item_rows": r["V"], "item_rows_per_gpu": r["rows_local"], "emb_dim": r["d"],
                       "parallelism": f"row-shard{world}" if world > 1 or FORCE_SHARD else "single",
                       "hipgraph": r["graphs"], "launch_mode": r["launch_mode"],
                       **({"collectives": r["collectives"]} if r.get("collectives") else {}),
                       **({"rehearsal": backend} if rehearsal else {}),
                       **({"launch_mode_trial_ms_per_step": r["mode_trial_ms_per_step"]}
                          if r.get("mode_trial_ms_per_step") else {}),
                       **({"batchnorm": "per-GPU statistics (nn.DataParallel semantics, train_fibinet.py:69-70)"
                           if args.bn == "local" else "SyncBN (global-batch statistics; the parity mode)"}
                          if world > 1 or FORCE_SHARD else {})},
            "host_enqueue_ms_per_step": round(r["t_host"] / K * 1e3, 4),
            **({"host_wait_ms_per_step": round(r["t_wait"] / K * 1e3, 4),
                "host_busy_ms_per_step": round((r["t_host"] - r["t_wait"]) / K * 1e3, 4)} if r["t_wait"] else {}),
            "roofline": r["roofline"],
            "rooflines": r["rooflines"],
            "rooflines_in_step_from": r["probe_source"],
            "table_adam": r["table_adam"],
            "steady_state": {"priming_steps": r["prime"], "warmup_steps": args.warmup,
                             "mean_replay_steps_per_claimed_row": round(r["lag"], 2),
                             "rows_touched_next_step": r["touched"],
                             "rows_replayed_on_critical_path": r["stale"],
                             "next_batch_prefetch": r["prefetch"],
                             "note": "untimed priming tops the warm-up up to 2F = 256 steps so the lazy "
                                     "table Adam is at steady state whatever --warmup is; with the next-batch "
                                     "prefetch the rows of step t+1 that step t does not touch are replayed on "
                                     "the side stream during step t (exact), so the claimed-row catch-up on the "
                                     "critical path replays only rows_replayed_on_critical_path rows"},
            "final_loss": round(r["loss"], 5),
        }
        if alt is not None:
            out["fp32"] = {"value": round(alt["K"] * B / alt["dt"], 1), "unit": "samples/s",
                           "ms_per_step": round(alt["dt"] / alt["K"] * 1e3, 4), "steps": alt["K"],
                           "process": alt.get("process", "bench"),
                           "roofline": alt["roofline"], "final_loss": round(alt["loss"], 5)}
        if alt16 is not None:
            out["c3_bf16_fwd"] = {
                "value": round(alt16["K"] * B / alt16["dt"], 1), "unit": "samples/s",
                "ms_per_step": round(alt16["dt"] / alt16["K"] * 1e3, 4), "steps": alt16["K"],
                "process": alt16.get("process", "bench"),
                "dtype": "bf16 forward GEMMs / fp32 backward",
                "gemm_precision": {"bf16 operands (fp32 accumulation)": [
                    "mm_proj x W_p", "bilinear U = V W", "MLP layer 1 c W_a", "MLP layer 2 h1 W_b"],
                    "fp32 operands as split-bf16 x3 (hi/lo images, A_hi B_hi + A_hi B_lo + A_lo B_hi, fp32 "
                    "accumulation; FBN_SPLIT3=0: fp32 MFMA)": [
                        "every backward GEMM: dh2 W_b, dW_b, dh1 W_a (dc), dW_a, dU W^T, dW, dW_p"],
                    "fp32": ["all non-GEMM arithmetic, master weights, Adam"]},
                # (its roofline counts the weight gradients' algorithmic flops once; the split runs three
                # bf16 MFMA products per fp32 one)
                "roofline": alt16["roofline"], "final_loss": round(alt16["loss"], 5)}
        if other_bn is not None:
            mode = "sync" if args.bn == "local" else "local"
            out["syncbn" if mode == "sync" else "local_bn"] = {
                "value": round(other_bn["K"] * B * world / other_bn["dt"], 1), "unit": "samples/s",
                "ms_per_step": round(other_bn["dt"] / other_bn["K"] * 1e3, 4), "steps": other_bn["K"],
                "batchnorm": ("SyncBN: statistics over the global batch -- the PARITY mode (one process on the "
                              "global batch); 4 extra all-reduces per step") if mode == "sync" else
                             "per-GPU statistics (nn.DataParallel semantics, train_fibinet.py:69-70)",
                "final_loss": round(other_bn["loss"], 5)}
        if ab is not None:
            out["native_ab"] = dict(ab, headline=(("native RCCL + step programs (validated bitwise against "
                                                   "torch.distributed)" if ab["validated"] else
                                                   "native RCCL + step programs (UNVALIDATED: the torch path failed)")
                                                  if native else "torch.distributed"),
                                    **({"native_headline_error": native_err} if native_err else {}))
        if torch_line is not None:
            out["torch_collectives"] = {
                "value": round(torch_line["K"] * B * world / torch_line["dt"], 1), "unit": "samples/s",
                "ms_per_step": round(torch_line["dt"] / torch_line["K"] * 1e3, 4), "steps": torch_line["K"],
                "launch_mode": torch_line["launch_mode"], "collectives": torch_line["collectives"],
                "host_enqueue_ms_per_step": round(torch_line["t_host"] / torch_line["K"] * 1e3, 4),
                "final_loss": round(torch_line["loss"], 5)}
        if inf is not None:
            out["inference"] = inf
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args, world)
            if args.cpu_plan:
                out["cpu_baseline_plan"] = cpu_baseline_plan(args)
        print(json.dumps(out), flush=True)
    if world > 1 or FORCE_SHARD:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
