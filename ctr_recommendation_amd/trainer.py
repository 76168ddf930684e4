"""Native fused FiBiNET training step on MI355X (single GPU or row-sharded over N GPUs).

Executes, per step, exactly what src/train_fibinet.py:113-123 does around the model:
  zero_grad -> forward -> BCELoss -> backward -> clip_grad_norm_(10) -> Adam(lr, wd) -> OneCycleLR
but as a sequence of libfibinet_hip.so launches with no host round trip (N = 1; capturable
into one hipGraph), and with the item-table gradient kept sparse:

* dense parameters (everything but the two id tables) live in ONE flat fp32 buffer with
  matching flat grad / Adam-m / Adam-v buffers: one norm pass and one fused Adam launch;
* the item-table gradient never exists as a dense V x d tensor.  The forward lets the first
  entry (sample, slot) that touches a row claim it (row -> entry map); the backward stores two
  vectors per sample (item-row and history-row gradients) with plain stores; a fix-up pass
  folds duplicate rows into their claimer; the dense Adam pass over the table reads the
  gradient of row r through the map (exact torch semantics: untouched rows still get
  g = wd * p) -- 24 B/element instead of zero-fill + scatter + 28 B/element;
* user_emb receives no gradient in the reference (the user field is zeros), so torch's Adam
  skips it; it is kept (state_dict contract) and never updated here either.

Multi-GPU (world > 1): one process per GPU; rows of E are block-sharded (exchange.py),
BatchNorm statistics are synchronised (SyncBN: the global-batch statistics the single-process
reference computes), dense gradients are all-reduced, the clip norm sums the table shards.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from . import _lib, ops
from ._lib import call, ptr
from .exchange import DistCollective, NativeComm, RowExchange, native_comm_wanted
from .model_fibinet import build_model

# single GPU, bf16: where the step's bf16 weight images are made (A/B knob) -- "main": on the
# main stream before the row claims; "side": on the side stream beside them; "late": on the side
# stream, captured after the claimed-row catch-up
_W16_MODE = os.environ.get("FBN_W16", "main")
# single GPU: the side-stream table-Adam passes (window + next-batch prefetch) forked after the
# MLP's first GEMM instead of right after the row claims (A/B knob)
_SIDE_AFTER_MLP0 = os.environ.get("FBN_SIDE_AFTER_MLP0", "0") == "1"
# ... or after the step's first GEMM (mm_proj), so a replayed graph launches that GEMM before the
# side-stream branch (A/B knob)
_SIDE_AFTER_MMPROJ = os.environ.get("FBN_SIDE_AFTER_MMPROJ", "0") == "1"
# single GPU, A/B knobs of the stream placement (tools/ab_step.py, in-process: each measured SLOWER
# than the default, profiles/r03_stream_placement_ab.txt):
#   FBN_CLAIM_ON_SIDE=1  the row claims + claimed-row catch-up on the side stream from the step's
#                        start, beside the bf16 weight images and the mm_proj GEMM (+15 us/step)
#   FBN_FIXUP_ON_SIDE=1  the duplicate-gradient fold on the side stream after the fields backward
#                        (round 3's first half: +2-3 us; since the weight gradients run as one grouped
#                        launch after the fields backward the fold hides beside it: 0.4290 vs 0.4321
#                        ms/step, profiles/r03s2_group_knobs_ab.txt -- so "auto", the default, puts it
#                        there whenever the side stream is in use)
#                        (+2-3 us/step)
#   FBN_SIDE_SERIAL=1    the rolling window + next-batch prefetch on the main stream, in sequence
#                        (0.5128 vs 0.4629 ms/step at C3: the overlap is worth 50 us there)
# FBN_SIDE_SERIAL defaults to "auto": in sequence on the main stream below d = 128, where the side
# work is small and the cross-queue edges cost more than the overlap saves (C2, graph-replayed:
# 0.2833-0.2844 vs 0.2934-0.2952 ms/step; eager 0.30 vs 0.45-0.50, the host's event waits gone;
# profiles/r03s2_side_serial_ab.txt), on the side stream from d = 128 on and in step programs
_CLAIM_ON_SIDE = os.environ.get("FBN_CLAIM_ON_SIDE", "0") == "1"
# single GPU, lazy table Adam, images on main: the bf16 image conversion rides in the row claims'
# launch (FBN_HEAD_CONV=0: its own launch ahead of the claims, A/B)
_HEAD_CONV = os.environ.get("FBN_HEAD_CONV", "1") != "0"
_SIDE_SERIAL = os.environ.get("FBN_SIDE_SERIAL", "auto")
# order of the side stream's two table-Adam passes (A/B knob): "wp" window then next-batch
# prefetch (default), "pw" the prefetch first, "p_w" the prefetch at the fork and the window only
# once the backward starts (the side stream waits for the forward)
_SIDE_ORDER = os.environ.get("FBN_SIDE_ORDER", "wp")
_FIXUP_ON_SIDE = os.environ.get("FBN_FIXUP_ON_SIDE", "auto")
# one join of the side stream per step after the fold (A/B knob: False joins again before the tail)
_JOIN_ONCE = True
# ... or after the gather (fields_fwd then runs with the chip to itself; A/B knob)
_SIDE_AFTER_GATHER = os.environ.get("FBN_SIDE_AFTER_GATHER", "0") == "1"
# N > 1: the next batch's routing enqueued after this step's compute (A/B knob)
_ROUTE_AFTER_COMPUTE = os.environ.get("FBN_ROUTE_AFTER_COMPUTE", "1") == "1"
# single GPU: the dense gradients' sum of squares inside the table-gradient norm launch (A/B knob)
_DENSE_SUMSQ_FOLD = os.environ.get("FBN_DENSE_SUMSQ_FOLD", "1") == "1"
# N > 1 (RCCL), opt-in (FBN_EARLY_GRAD_XCHG=1): the gradient-row all-to-all issued right after the
# fields backward and the dense-gradient all-reduce right after the compute, both asynchronous on
# the process group's stream beside the remaining work (the loss + table sum of squares then take
# a small all-reduce of their own).  Off by default: as a one-rank RCCL job it measured 0.73-0.74
# vs 0.69-0.72 ms/step (extra launches, a local-copy "all-to-all" competing for HBM) and the
# overlap it buys at N > 1 could not be measured on a one-GPU box
_EARLY_GRAD_XCHG = os.environ.get("FBN_EARLY_GRAD_XCHG")
# single GPU, eager steps with the side stream (A/B knob, FBN_WGRAD_EARLY=1): the grouped weight-
# gradient GEMMs of the MLP and the bilinear W (dWa, dWb, dW) launched on the side stream right after
# the bilinear backward, beside the fields backward (HBM-bound) on the main stream; dW_p stays in the
# flush's launch on main, which waits for the side stream before the slab sums
_WGRAD_EARLY = os.environ.get("FBN_WGRAD_EARLY", "0") == "1"
# single GPU, d >= 128, A/B knob FBN_PF_BINNED=1: the next-batch prefetch's replay balanced longest-first
# (fbn_adam_prefetch_binned).  Bit-identical, measured slower (0.443 vs 0.421 ms/step at C3),
# so adam_prefetch2's 64-entries-per-wave replay stays the default
_PF_BINNED = os.environ.get("FBN_PF_BINNED", "0") == "1"
# N > 1 (and the one-rank sharded run): the fixed-capacity exchange (RowExchange.enable_fixed) once
# FC_CALIB_STEPS steps measured the per-owner load -- equal-split all-to-alls, no host-side split
# sizes, the step recordable as a step program.  FBN_FC=0 keeps the host-split exchange (A/B);
# FBN_FC_CAP=<n> fixes the per-block capacity instead of calibrating it; FBN_FC_MARGIN (1.25) scales
# the calibrated load
_FC = os.environ.get("FBN_FC", "1") != "0"
_FC_CAP = int(os.environ.get("FBN_FC_CAP", "0"))
_FC_MARGIN = float(os.environ.get("FBN_FC_MARGIN", "1.25"))
FC_CALIB_STEPS = 2
FBN_GRAD_CELL = 0x20000      # include/fibinet.h: the gradient-row argument is a device cell (fbn_ring_slot)
FBN_GRAD_BF16 = 0x40000      # include/fibinet.h: the per-entry gradient rows are bf16
FBN_RING_BF16 = 0x40000000   # include/fibinet.h: ring_n flag, the deferred-gradient ring holds bf16 rows
# N > 1 in bf16 mode, opt-in (FBN_RING_BF16=1): the owner's deferred-gradient ring keeps the wire's bf16
# gradient rows as they arrive (the fold copies them instead of widening them to f32: half the ring's
# bytes written per step and read per replayed row; the same f32 values on every read -- bitwise equal,
# tests/test_gpu_rccl.py).  Measured no faster at one rank (0.4825 vs 0.4787 ms/step), so
# the f32 ring stays the default
_RING_BF16 = os.environ.get("FBN_RING_BF16", "0") == "1"
# N > 1, the owner's ahead-of-time catch-up of the next step's requested rows in two passes (tagged
# pre-claims + the four-row replay engine); FBN_OWNER_PF2=0 keeps the one-pass kernel (A/B)
_OWNER_PF2 = os.environ.get("FBN_OWNER_PF2", "1") != "0"
# N > 1, the fixed-capacity exchange: the owner's claims and claimed-row catch-up in one launch
# (fbn_adam_owner_claim_catchup, pre-claims from the owner prefetch); FBN_OWNER_CLAIM_FUSED=0 keeps
# fbn_owner_claim + fbn_adam_catchup (A/B)
_OWNER_CLAIM_FUSED = os.environ.get("FBN_OWNER_CLAIM_FUSED", "1") != "0"
# ... and the widen into the ring slot + the duplicate fold in one pass (fbn_owner_fold; duplicates
# summed in extra[claimer], applied at the tail); FBN_OWNER_FOLD=0 keeps fbn_ring_slot +
# fbn_sparse_fixup (A/B)
_SHARD_W16_SIDE = os.environ.get("FBN_SHARD_W16_SIDE", "1") != "0"
_OWNER_FOLD = os.environ.get("FBN_OWNER_FOLD", "1") != "0"
# debug: after every record_program, check that no tensor of the trainer's persistent state lies in the
# recording pool (check_program_memory; the tests run it explicitly)
_CHECK_POOL = os.environ.get("FBN_CHECK_POOL", "0") == "1"
from .schedule import OneCycle, adam_table

TABLE = "item_emb.weight"
FBN_GRAD_FULL = 0x10000      # include/fibinet.h: extra holds the full row gradient (deterministic fold)
FROZEN = ("user_emb.weight",)
BUFFERS = ("mlp.1.running_mean", "mlp.1.running_var", "mlp.1.num_batches_tracked",
           "mlp.5.running_mean", "mlp.5.running_var", "mlp.5.num_batches_tracked")


def _events(probe, name, stream=None):
    """Arm a kernel-span probe (_lib.KernelProbe) for the next library call, recorded under `name`
    (bench probes); _events_end() right after that call."""
    if probe is None:
        return None
    kp = _lib.KernelProbe()
    probe.setdefault(name, []).append((kp, None))
    return kp


def _events_end(kp, stream=None):
    if kp is not None:
        kp.done()


def default_lazy_window(d: int) -> int:
    """The rolling window F of the lazy table Adam (every row is visited at least once per F steps;
    the deferred-gradient ring holds F + 1 steps).  The window pass is bound by its longest replay
    chain (lags up to F), not by its rows: at C3 (d = 128) F = 128 measured best (64 / 32: +9 / +22
    us per step), at C2 (d = 16, the side passes in sequence on the main stream) F = 32 (0.264 vs
    0.287 ms/step at 128; 16 / 8 within noise of 32) -- profiles/r03s2_lazy_window_sweep.txt."""
    return 128 if d >= 128 else 32


def _side_stream(dev):
    """The side stream; FBN_SIDE_CU_MASK=<hex word>[,<hex word>...] (32 CUs per word, repeated to
    cover the device) restricts it to a CU subset (hipExtStreamCreateWithCUMask) -- tuning knob
    (measured: restricting the table-Adam side work to 64 or 32 CUs doubles the step time)."""
    mask = os.environ.get("FBN_SIDE_CU_MASK")
    if not mask:
        return torch.cuda.Stream(device=dev)
    words = [int(w, 16) for w in mask.split(",")]
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    n = (ncu + 31) // 32
    arr = (ctypes.c_uint32 * n)(*[words[i % len(words)] for i in range(n)])
    hip = ctypes.CDLL("libamdhip64.so")
    s = ctypes.c_void_p()
    with torch.cuda.device(dev):
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), n, arr)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({rc})")
    return torch.cuda.ExternalStream(s.value, device=dev)


class _Segments:
    """The collective hook of a captured compute region: ops.forward / ops.backward run once
    under capture with this object as their `coll`; every allreduce_ (the SyncBN moments) closes
    the hipGraph segment being captured and opens the next, so a replay is segment, all-reduce,
    segment, ... -- the all-reduces stay eager RCCL calls with host-side arguments (nothing
    collective is captured), the ~45 kernel launches between them become a handful of graph
    launches."""

    def __init__(self, base, pool):
        self.base, self.world, self.pool = base, base.world, pool
        self.prog: list = []
        self.cur = None

    def begin(self) -> None:
        self.cur = torch.cuda.CUDAGraph()
        # thread-local: the process group's watchdog thread keeps querying its events meanwhile
        self.cur.capture_begin(pool=self.pool, capture_error_mode="thread_local")

    def allreduce_(self, t: torch.Tensor) -> None:
        self.cur.capture_end()
        self.prog += [("graph", self.cur), ("allreduce", t)]
        self.begin()

    def call(self, fn) -> None:
        """Close the segment; a replay runs fn() (host code: e.g. an asynchronous collective) here."""
        self.cur.capture_end()
        self.prog += [("graph", self.cur), ("call", fn)]
        self.begin()

    def end(self) -> None:
        self.cur.capture_end()
        self.prog.append(("graph", self.cur))
        self.cur = None

    def replay(self) -> None:
        for kind, x in self.prog:
            if kind == "graph":
                x.replay()
            elif kind == "call":
                x()
            else:
                self.base.allreduce_(x)


def _copy_many(pairs, stream) -> None:
    """dst.copy_(src) for every (src, dst) pair, same shapes and dtypes: the 16-byte-aligned
    contiguous ones in fbn_copy_jobs launches of up to 8, any other with copy_."""
    fused = []
    for src, dst in pairs:
        nb = src.numel() * src.element_size()
        if (src.is_contiguous() and dst.is_contiguous() and nb % 16 == 0 and src.data_ptr() % 16 == 0
                and dst.data_ptr() % 16 == 0):
            fused.append((src.data_ptr(), dst.data_ptr(), nb))
        else:
            dst.copy_(src, non_blocking=True)
    for i in range(0, len(fused), 8):
        chunk = fused[i:i + 8]
        n = len(chunk)
        call("fbn_copy_jobs", (ctypes.c_void_p * n)(*[c[0] for c in chunk]),
             (ctypes.c_void_p * n)(*[c[1] for c in chunk]), (ctypes.c_longlong * n)(*[c[2] for c in chunk]), n,
             stream)


def _batch_key(item: torch.Tensor, seq: Optional[torch.Tensor]):
    """Identity of a batch's id tensors for work prepared one step ahead (pre-claims, routing):
    address, shape AND version counter, so a caller that copies the next batch into the same
    static buffer (copy_ bumps _version) gets a fresh claim instead of the previous batch's."""
    return (item.data_ptr(), item.shape[0], item._version,
            0 if seq is None else seq.data_ptr(), 0 if seq is None else tuple(seq.shape),
            0 if seq is None else seq._version)


def _lib_key(x, batch):
    """RowExchange's routing key of a batch (the id tensors, their shapes and version counters)."""
    seq = batch.get("item_seq")
    return x._key(batch["item_id"], seq if seq is not None and seq.shape[1] else None)


def _pad4(n: int) -> int:
    return (n + 3) // 4 * 4


class FiBiNETTrainer:
    def __init__(self, model_cfg: Dict, total_steps: int, batch_size: int, *, device=None, max_len: int = 20,
                 lr: Optional[float] = None, weight_decay: Optional[float] = None, rank: int = 0, world: int = 1,
                 group=None, init_state: Optional[Dict[str, torch.Tensor]] = None, seed: int = 2025,
                 stage_on_cpu: bool = False, dropout_seed: Optional[int] = None, table_adam: str = "lazy",
                 lazy_window: Optional[int] = None, defer_table_grads: bool = True, max_norm: float = 10.0,
                 optimizer: Optional[str] = None, deterministic: Optional[bool] = None,
                 prefetch_rows: bool = True, shard: Optional[bool] = None, sync_bn: Optional[bool] = None,
                 native_comm: Optional[bool] = None):
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise RuntimeError("FiBiNETTrainer runs on a HIP device only (no CPU fallback)")
        self.cfg = dict(model_cfg)
        self.lr = float(lr if lr is not None else model_cfg.get("learning_rate", 1e-3))
        self.wd = float(weight_decay if weight_decay is not None else model_cfg.get("weight_decay", 1e-5))
        # clip_grad_norm_(model.parameters(), max_norm=10.0) (train_fibinet.py:119); settable so
        # tests can make the clip engage
        self.beta2, self.eps, self.max_norm = 0.999, 1e-8, float(max_norm)
        # torch.optim.Adam with coupled L2 (train_fibinet.py:78) -- the reference's code; the config's
        # `optimizer: adamw` (fibinet_config.yaml:62) is dead there and honoured only on request
        # (honour_config, or optimizer="adamw"): torch.optim.AdamW's decoupled decay, opt-in, non-parity
        honour = bool(model_cfg.get("honour_config", False))
        opt = optimizer or (str(model_cfg.get("optimizer", "adam")) if honour else "adam")
        if opt.lower() not in ("adam", "adamw"):
            raise ValueError(f"optimizer must be 'adam' or 'adamw', not {opt!r}")
        self.optimizer = opt.lower()
        self.decoupled = self.optimizer == "adamw"
        self.wd_g = 0.0 if self.decoupled else self.wd           # weight decay inside the gradient
        self.rank, self.world, self.group = rank, world, group
        # the row-sharded path (exchange, owner-side table Adam); shard=True runs it at world = 1 too
        # (an RCCL smoke test of the N > 1 code on a one-GPU box: every collective has one rank)
        self.sharded = world > 1 if shard is None else bool(shard)
        sharded = self.sharded
        self.B = batch_size                     # per-rank batch
        self.L = max_len
        if init_state is None:
            torch.manual_seed(seed)
            init_state = build_model(None, self.cfg).state_dict()
        with torch.random.fork_rng(devices=[]):            # no side effect on the caller's RNG stream
            shape_model = build_model(None, dict(self.cfg, vocab_size=4))
        self.key_order = list(shape_model.state_dict().keys())
        self.d = shape_model.emb_dim
        self.p_drop = shape_model.dropout_p
        self.fcfg = ops.FwdConfig(d=self.d, L=max_len, training=True, p_drop=self.p_drop,
                                  bf16=shape_model.compute_bf16, fwd16=shape_model.compute_fwd16,
                                  bilinear_each=shape_model.bilinear.bilinear_type == "each",
                                  R=shape_model.senet.excitation[0].out_features)
        self.V = init_state[TABLE].shape[0]
        dev = self.device
        d = self.d
        # ---------------- dense parameters: one flat buffer (16-B aligned segments)
        self.dense_names: List[str] = [n for n, _ in shape_model.named_parameters() if n != TABLE and n not in FROZEN]
        self.shapes = {n: tuple(init_state[n].shape) for n in self.key_order}
        offs, o = {}, 0
        for n in self.dense_names:
            offs[n] = o
            o += _pad4(int(np.prod(self.shapes[n])))
        self.n_dense = o
        self.flat_p = torch.zeros(o, dtype=torch.float32, device=dev)
        # dense grads + 2 trailing floats (loss, table sumsq) for the multi-GPU all-reduce
        self.flat_g_ext = torch.zeros(o + 4, dtype=torch.float32, device=dev)
        self.flat_g = self.flat_g_ext[:o]
        self.flat_m = torch.zeros_like(self.flat_p)
        self.flat_v = torch.zeros_like(self.flat_p)
        self.p: Dict[str, torch.Tensor] = {}
        self.g: Dict[str, torch.Tensor] = {}
        for n in self.dense_names:
            k = int(np.prod(self.shapes[n]))
            self.p[n] = self.flat_p[offs[n]:offs[n] + k].view(self.shapes[n])
            self.g[n] = self.flat_g[offs[n]:offs[n] + k].view(self.shapes[n])
            self.p[n].copy_(init_state[n].to(dev))
        for n in FROZEN:
            self.p[n] = init_state[n].to(dev).clone()
        for n in BUFFERS:
            self.p[n] = init_state[n].to(dev).clone()
        # ---------------- item table shard + Adam state + sparse gradient bookkeeping
        self.Vl = (self.V + world - 1) // world
        lo = rank * self.Vl
        hi = min(self.V, lo + self.Vl)
        self.rows_lo, self.rows_local = lo, hi - lo
        self.E = init_state[TABLE][lo:hi].to(dev).contiguous()
        self.Em = torch.zeros_like(self.E)
        self.Ev = torch.zeros_like(self.E)
        if world == 1:
            self.p[TABLE] = self.E
        i32 = dict(dtype=torch.int32, device=dev)
        self.n_entries = self.B * (max_len + 1) if not sharded else world * self.B * (max_len + 1)
        self.map = torch.full((max(1, self.rows_local),), -1, **i32)         # row -> claiming entry
        self.slot_row = torch.full((self.n_entries,), -1, **i32)              # entry -> claimed row
        self.gvec = torch.zeros((self.B, 2, d), dtype=torch.float32, device=dev) if not sharded else None
        self.extra = torch.zeros((self.n_entries, d), dtype=torch.float32, device=dev) if not sharded else None
        # single GPU: claim-time duplicate list (entry -> claiming entry) and per-sample gradient norms
        self.dup = torch.full((self.n_entries,), -1, **i32) if not sharded else None
        self.gnorm = torch.zeros((self.B, 2), dtype=torch.float64, device=dev) if not sharded else None
        # deterministic mode (src/utils.py:15-16): rows hit by several entries are folded by
        # order-independent int64 fixed-point sums instead of float atomics -- single GPU
        # fbn_sparse_fold_fx, the sharded owner fbn_owner_fold(fx) + fbn_sumsq_flagged(fx) -- so two runs
        # from the same state produce bit-identical table gradients and weights (and a one-rank sharded
        # run the single-GPU run's)
        if deterministic is None:
            deterministic = bool(model_cfg.get("deterministic", False)) or os.environ.get("FBN_DETERMINISTIC") == "1"
        self.deterministic = bool(deterministic)
        self._fx_sh = None          # sharded deterministic fold: fixed-point accumulator [n][d] (zero at rest)
        # lazy table Adam, single GPU: step(..., next_batch=...) brings the next batch's rows up to
        # date on the side stream during this step (fbn_adam_prefetch; d < 128 needs the next batch
        # to have this batch's shape -- its pre-claims drive the two-pass form)
        self.prefetch_rows = bool(prefetch_rows) and not sharded and self.d in (16, 32, 64, 128, 256)
        # N > 1, the owner's side: the next step's requested rows arrive during this step (the
        # padded id exchange of RowExchange.prepare) and are caught up ahead (fbn_adam_prefetch_rows)
        self.prefetch_owner = bool(prefetch_rows) and sharded and self.d in (128, 256)
        # the prefetch also decides the next batch's row claims (tagged, no CAS at claim time);
        # they are used only by a step given the very id tensors they were made for
        # per-row table-Adam state: ONE 16-B record per row {i64 pre-claim tag, i32 last, i32 pend}
        # (include/fibinet.h FBN_ROW_STATE_BYTES); .preclaim / .last / .pend are strided views of it
        self.row_state = torch.zeros((max(1, self.rows_local), 4), **i32)
        self.row_state[:, 3] = -1
        self.preclaim = self.row_state.view(torch.int64)[:, 0] if self.prefetch_rows else None
        # scratch of the binned prefetch (bins of replay records), d >= 128
        self.pf_ws = None
        if self.prefetch_rows and self.d >= 128:
            nb = _lib.lib().fbn_adam_prefetch_binned_ws_size(self.B * (max_len + 1))
            self.pf_ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        self._pre_key = None
        self.hasdup = torch.zeros((self.n_entries,), **i32) if self.deterministic and not sharded else None
        self.fx = torch.zeros((self.n_entries, d), dtype=torch.int64, device=dev) \
            if self.deterministic and not sharded else None
        # ---------------- optimizer schedule + device step state
        self.total_steps = total_steps
        tab, self.lrs = adam_table(total_steps, self.lr, self.beta2, OneCycle(total_steps, self.lr),
                                   decoupled_wd=self.wd if self.decoupled else 0.0)
        self.sched = torch.from_numpy(tab).to(dev)
        self.step_dev = torch.zeros(1, **i32)
        seed_d = dropout_seed if dropout_seed is not None else (seed * 1000003 + 17)
        seed_d += rank * 0x9E3779B9            # independent dropout stream per rank
        self.rng = torch.tensor([seed_d & 0x7FFFFFFFFFFF, 0], dtype=torch.int64, device=dev)
        self.sumsq = torch.zeros(64, dtype=torch.float64, device=dev)        # FBN_SUMSQ_SLOTS
        self.sumsq_tab = torch.zeros(64, dtype=torch.float64, device=dev)
        self.coef = torch.ones(1, dtype=torch.float32, device=dev)
        self.norm = torch.zeros(1, dtype=torch.float32, device=dev)
        self.err = torch.zeros(1, **i32)
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self.host_step = 0
        self.acts: Dict[str, torch.Tensor] = {}
        # RCCL on the step's own stream (exchange.NativeComm) when the process group is RCCL
        # (native_comm: True / False overrides FBN_NATIVE_COMM -- bench.py's lockstep A/B of the two paths)
        self.native_comm = NativeComm(world, rank, group, dev) \
            if (sharded or world > 1) and native_comm_wanted(dev, group, stage_on_cpu, force=native_comm) else None
        # (deterministic mode: the all-reduces as all-gather + rank-ordered sums, bitwise reproducible)
        self.coll = DistCollective(world, group, stage_on_cpu, comm=self.native_comm, det=self.deterministic)
        # BatchNorm at N > 1.  sync_bn (default): statistics over the GLOBAL batch (one f64
        # all-reduce per BN layer and direction) -- the single-process reference run on the
        # global batch.  sync_bn=False: every rank normalises its own slice, which is what the
        # reference script itself does on a multi-GPU box (nn.DataParallel, train_fibinet.py:69-70:
        # each replica's BatchNorm1d sees its scattered slice; running statistics survive from the
        # device-0 replica only -> here each rank keeps its own and rank 0's are checkpointed).
        # No collective inside the forward / backward then: the captured compute is ONE segment.
        self.sync_bn = bool(model_cfg.get("sync_bn", True) if sync_bn is None else sync_bn)
        self.bn_coll = self.coll if self.sync_bn else ops.NO_COLLECTIVE
        self.side = _side_stream(dev)      # eager untouched pass / lazy rolling window / routing ahead
        self.xchg = RowExchange(rank, world, self.V, d, self.B, max_len, dev, group, stage_on_cpu=stage_on_cpu,
                                rows_bf16=self.fcfg.bf16, side=self.side, comm=self.native_comm) if sharded else None
        self.stage_on_cpu = stage_on_cpu
        self.early_grad_xchg = _EARLY_GRAD_XCHG == "1"
        # item-table Adam: "lazy" (default) replays the zero-gradient steps of a row when the row
        # is next claimed or its rolling window comes round (bit-identical to eager; see
        # fbn_adam_catchup) -- "eager" streams every untouched row each step on a side stream (the
        # reference's dense update order, kept for A/B measurements) -- "sparse" (opt-in,
        # NON-parity, for 100M-row tables): only the rows a batch touches are updated, as
        # torch.optim.SparseAdam does (plus the coupled L2 term on those rows); untouched rows,
        # their moments included, stay frozen
        self.table_adam = os.environ.get("FBN_TABLE_ADAM", table_adam)
        if self.table_adam not in ("lazy", "eager", "sparse"):
            raise ValueError(f"table_adam must be 'lazy', 'eager' or 'sparse', not {self.table_adam!r}")
        self.lazy_window = int(lazy_window) if lazy_window is not None else default_lazy_window(d)
        # single GPU: the side-stream table-Adam passes in sequence on the main stream (see _SIDE_SERIAL)
        self.side_serial = _SIDE_SERIAL == "1" or (_SIDE_SERIAL == "auto" and d < 128)
        self.last = self.row_state[:, 2]     # Adam steps applied per table row
        # lazy: deferred table gradients (the step tail's commit) -- pend[r] = the gradient row r
        # received at step last[r], applied at the row's next replay; the last F+1 steps' gradients
        # stay in a ring: single GPU, the per-sample vectors [B][2][d]; N > 1, the owner's received
        # per-entry rows, up to ring_cap per step (a step receiving more applies its rows at once)
        self.deferred = self.table_adam == "lazy" and defer_table_grads
        self.pend = self.ring = self.coef_hist = None
        self.ring_n = self.lazy_window + 1
        self.ring_cap = self.B * (max_len + 1) if sharded else 0
        # sharded bf16 mode: a bf16 ring (the wire's rows as they arrived; _RING_BF16)
        self.ring_bf16 = bool(sharded and self.fcfg.bf16 and _RING_BF16 and self.deferred)
        if self.deferred:
            self.pend = self.row_state[:, 3]
            shape = (self.ring_n, self.B, 2, d) if not sharded else (self.ring_n, self.ring_cap, d)
            self.ring = self._new_ring(shape)
            self.coef_hist = torch.ones(total_steps + 1, dtype=torch.float32, device=dev)
            self.ticket = torch.zeros(17, dtype=torch.int32, device=dev)    # fbn_adam_step_tail (FBN_TICKET_WORDS)
        # N > 1: forward + backward between the row exchanges replayed as hipGraph segments split at
        # the SyncBN all-reduces (_Segments), after two eager steps; FBN_SHARD_GRAPH=0 keeps it eager
        self.shard_graph = self.sharded and os.environ.get("FBN_SHARD_GRAPH", "1") != "0"
        self._late_side = None
        self._sg = None
        self._sg_eager = 0
        self._bn_synced_at = -1     # host step of the last rank-0 BatchNorm broadcast (_bn_from_rank0)
        self._used_pre = False      # the last step took its row claims from the prefetch's pre-claims
        self._recording = False     # inside record_program()
        # fixed-capacity exchange: calibration (largest per-owner block seen) and the ring-slot cell
        self.fc_wanted = self.sharded and _FC and self.device.type == "cuda"
        self._fc_seen = 0
        self._fc_steps = 0
        self.ring_cell = torch.zeros(2, dtype=torch.int64, device=dev)     # fbn_ring_slot's pointer cell
        self._fc_grad = None        # fixed-capacity rows, f32, when they are not deferred
        self._fc_extra = None       # fixed-capacity form: duplicates' sums per claimer (zero at rest)
        self._fc_part = None        # ... and fbn_owner_fold's per-workgroup sums of squares

    # ------------------------------------------------------------------ one training step
    def step(self, batch: Dict[str, torch.Tensor], labels: torch.Tensor,
             masks_out: Optional[Dict[str, torch.Tensor]] = None, probe: Optional[Dict[str, list]] = None,
             next_batch: Optional[Dict[str, torch.Tensor]] = None) -> torch.Tensor:
        """One optimizer step on this rank's batch; returns the (device) global-mean BCE loss.

        masks_out (tests only): {'m1': u8 [B,512], 'm2': u8 [B,256]} receives the dropout keep-masks.
        probe (bench only): collects HIP-event pairs around the gather and table-Adam launches.
        next_batch: the batch of the FOLLOWING step.  N > 1: its ids are routed and their counts
        exchanged during this step on a side stream (RowExchange.prepare), so the next step needs
        no host sync on the main stream; that step uses the routing only if it is given the very
        same id tensors (unmodified), otherwise it routes inline.  N = 1 (lazy table Adam, d = 128
        / 256): its rows that this batch does not touch are brought up to date on the side stream
        now (fbn_adam_prefetch) -- exact whatever batch the next step actually gets.
        """
        if self.host_step >= self.total_steps:
            raise ValueError(f"Tried to step {self.host_step + 1} times. The specified number of total steps is "
                             f"{self.total_steps}")
        st = _lib.stream_handle(self.device)
        B = batch["item_id"].shape[0]
        if B > self.B:
            raise ValueError(f"batch of {B} rows exceeds the trainer's batch_size {self.B}")
        ntot = B * self.world
        d = self.d
        cfg = self.fcfg
        seq = batch.get("item_seq")
        L = cfg.L = seq.shape[1] if seq is not None else 0
        if L > self.L:
            raise ValueError(f"history length {L} exceeds max_len {self.L}")
        rows = pos = None
        main = torch.cuda.current_stream(self.device)

        lazy = self.table_adam == "lazy"

        side_hooks = {}

        def catch_up(n_ent, claim=False, before_side=None, on_side=None):
            # lazy table Adam: the rows claimed this step are brought to `step` Adam steps before
            # anything reads them; the rolling window (step % F; unclaimed rows, read by nothing
            # this step) replays on the side stream beside the rest of the step.  claim (single
            # GPU): the row claims are made inside the same launch (fbn_adam_claim_catchup).
            # on_side (an event on main at the step's start): the claims run on the side stream,
            # and the main stream waits for them just before the gather
            if on_side is not None:
                _lib.wait_event(self.side, on_side)
                ev = _events(probe, "adam_catchup", self.side)
                key = _batch_key(batch["item_id"], seq if L else None)
                pre = self.preclaim if (self.preclaim is not None and key == self._pre_key) else None
                self._used_pre = pre is not None
                self._pre_key = None
                call("fbn_adam_claim_catchup", ptr(batch["item_id"]), ptr(seq) if L else None, B, L, self.V,
                     ptr(self.map), ptr(self.slot_row), ptr(self.dup), ptr(self.hasdup), ptr(pre), ptr(self.E),
                     ptr(self.Em), ptr(self.Ev), self.rows_local, d, self.lazy_window, ptr(self.last),
                     ptr(self.sched), ptr(self.step_dev), self.wd_g, self.beta2, self.eps, *self._pend_args(),
                     int(self.decoupled), self.side.cuda_stream)
                _events_end(ev, self.side)
                claim_ev = torch.cuda.Event()
                _lib.record_event(claim_ev, self.side)
                side_hooks["before_gather"] = lambda: _lib.wait_event(main, claim_ev)
                side_pass(wait_main=False)
                return
            ev = _events(probe, "adam_catchup")
            if claim:
                key = _batch_key(batch["item_id"], seq if L else None)
                pre = self.preclaim if (self.preclaim is not None and key == self._pre_key) else None
                self._used_pre = pre is not None
                self._pre_key = None
                args = (ptr(batch["item_id"]), ptr(seq) if L else None, B, L, self.V, ptr(self.map),
                        ptr(self.slot_row), ptr(self.dup), ptr(self.hasdup), ptr(pre), ptr(self.E), ptr(self.Em),
                        ptr(self.Ev), self.rows_local, d, self.lazy_window, ptr(self.last), ptr(self.sched),
                        ptr(self.step_dev), self.wd_g, self.beta2, self.eps, *self._pend_args(), int(self.decoupled))
                if head_conv:
                    # the step head: the bf16 images converted in the same launch as the claims
                    call("fbn_adam_claim_catchup_conv", *args, *head_conv, st)
                else:
                    call("fbn_adam_claim_catchup", *args, st)
            else:
                call("fbn_adam_catchup", ptr(self.E), ptr(self.Em), ptr(self.Ev), self.rows_local, d,
                     ptr(self.slot_row), n_ent, ptr(self.map), self.lazy_window, 1, ptr(self.last), ptr(self.sched),
                     ptr(self.step_dev), self.wd_g, self.beta2, self.eps, *self._pend_args(), int(self.decoupled), st)
            _events_end(ev)
            if before_side is not None:
                self._w16_ev = start_w16(before_side)   # the side stream: images first, then the window
            if claim and _SIDE_AFTER_MLP0:
                side_hooks["after_mlp0"] = side_pass     # forked after the MLP's first GEMM instead
                return
            if claim and _SIDE_AFTER_MMPROJ:
                side_hooks["after_mmproj"] = side_pass   # forked after the step's first GEMM
                return
            if claim and _SIDE_AFTER_GATHER:
                side_hooks["after_fields"] = side_pass   # forked after the gather
                return
            side_pass()

        def side_pass(wait_main=True):
            # a step being recorded as a step program runs its side passes on the side stream at every
            # d: replayed natively, the two edges cost less than the overlap saves (C2: 0.2071-0.2082
            # vs 0.2176-0.2190 ms/step, profiles/r04_c2_stream_placement.txt)
            serial = self.side_serial and not (self._recording and _SIDE_SERIAL == "auto")
            sst = self.side if not serial else main      # in sequence on main (FBN_SIDE_SERIAL)
            if wait_main and not serial:
                _lib.wait_stream(self.side, main)

            def window():
                ev = _events(probe, "adam_window", sst)
                call("fbn_adam_catchup", ptr(self.E), ptr(self.Em), ptr(self.Ev), self.rows_local, d, None, 0,
                     ptr(self.map), self.lazy_window, 2, ptr(self.last), ptr(self.sched), ptr(self.step_dev),
                     self.wd_g, self.beta2, self.eps, *self._pend_args(), int(self.decoupled), sst.cuda_stream)
                _events_end(ev, sst)

            order = _SIDE_ORDER if not serial else "wp"
            if order == "wp":
                window()
            prefetch_pass(sst)
            if order == "pw":
                window()
            elif order == "p_w":
                def late_window():
                    _lib.wait_stream(self.side, main)      # the forward is done: the window beside the backward
                    window()
                self._late_side = late_window

        def prefetch_pass(sst):
            nb = next_batch
            if (self.xchg is None and nb is not None and self.prefetch_rows and nb["item_id"].dtype == torch.int64
                    and nb["item_id"].device == self.device):
                nseq = nb.get("item_seq")
                nL = nseq.shape[1] if nseq is not None else 0
                if nb["item_id"].shape[0] == B and nL == L:   # claims made now are valid for that step
                    self._pre_key = _batch_key(nb["item_id"], nseq if nL else None)
                elif d < 128:
                    return                                    # the one-pass form needs wave-wide rows
                ev = _events(probe, "adam_prefetch", sst)
                nB = nb["item_id"].shape[0]
                if (_PF_BINNED and self._pre_key is not None and self.pf_ws is not None
                        and nB * (nL + 1) <= self.B * (self.L + 1)):
                    call("fbn_adam_prefetch_binned", ptr(nb["item_id"]), ptr(nseq) if nL else None, nB, nL,
                         self.V, ptr(self.map), ptr(self.preclaim), ptr(self.E), ptr(self.Em), ptr(self.Ev), d,
                         ptr(self.last), ptr(self.sched), ptr(self.step_dev), self.wd_g, self.beta2, self.eps,
                         *self._pend_args(), int(self.decoupled), ptr(self.pf_ws), self.pf_ws.numel(),
                         sst.cuda_stream)
                    _events_end(ev, sst)
                    return
                call("fbn_adam_prefetch", ptr(nb["item_id"]), ptr(nseq) if nL else None, nB, nL,
                     self.V, ptr(self.map), ptr(self.preclaim if self._pre_key is not None else None), ptr(self.E),
                     ptr(self.Em), ptr(self.Ev), d, ptr(self.last),
                     ptr(self.sched), ptr(self.step_dev), self.wd_g, self.beta2, self.eps, *self._pend_args(),
                     int(self.decoupled), sst.cuda_stream)
                _events_end(ev, sst)

        def start_untouched_adam():
            # eager mode: every row this shard's batch does not touch gets g = wd * p, independent
            # of the backward -> concurrently on the side stream
            _lib.wait_stream(self.side, main)
            ev = _events(probe, "adam_table", self.side)
            call("fbn_adam_table", ptr(self.E), ptr(self.Em), ptr(self.Ev), self.rows_local, d, ptr(self.map),
                 None, None, None, 1, None, ptr(self.sched), ptr(self.step_dev), self.wd_g, self.beta2, self.eps, 1,
                 self.side.cuda_stream)
            _events_end(ev, self.side)

        w16_ev = None

        def start_w16(after=None):
            # bf16 weight images (they depend only on the weights the previous step wrote) on the side
            # stream, beside the row claims and the claimed-row catch-up
            if after is None:
                _lib.wait_stream(self.side, main)
            else:
                _lib.wait_event(self.side, after)
            with torch.cuda.stream(self.side):
                self.acts["w16"] = ops.bf16_weights(self.p, d, self.acts, self.side.cuda_stream,
                                                    x=batch["item_emb_d128"])
            ev = torch.cuda.Event()
            _lib.record_event(ev, self.side)
            return ev

        # bf16_fwd training on the split-bf16 x3 backward: the forward's weight images (and their lo
        # images) made here too, in the claims' launch, instead of at the forward's start
        w16_img = bool(cfg.fwd16 and not cfg.bf16 and ops._SPLIT3 and not cfg.bilinear_each and cfg.training)
        w16_main = (cfg.bf16 or w16_img) and self.xchg is None and _W16_MODE == "main"
        self.acts["w16_images"] = w16_main and w16_img
        w16_late = cfg.bf16 and self.xchg is None and lazy and _W16_MODE == "late"
        claim_side = None
        if (self.xchg is None and lazy and _CLAIM_ON_SIDE and not w16_late and not _SIDE_AFTER_MLP0
                and not _SIDE_AFTER_MMPROJ and not _SIDE_AFTER_GATHER):
            claim_side = torch.cuda.Event()          # the step's start: the claims wait for nothing later
            _lib.record_event(claim_side, main)
        head_conv = None
        if w16_main and self.xchg is None and lazy and claim_side is None and _HEAD_CONV:
            # on the main stream, in the claims' launch (fbn_adam_claim_catchup_conv): the two are
            # independent, so they run side by side instead of one launch after the other
            jobs, njobs, self.acts["w16"] = ops.bf16_weight_jobs(self.p, d, self.acts, x=batch["item_emb_d128"],
                                                                 images=w16_img)
            head_conv = (ctypes.cast(jobs, ctypes.c_void_p).value, njobs)
        elif w16_main:
            # on the main stream ahead of the claims: a cross-queue wait inside a replayed graph
            # costs ~10 us, about what the conversion itself takes
            self.acts["w16"] = ops.bf16_weights(self.p, d, self.acts, st, x=batch["item_emb_d128"], images=w16_img)
        elif cfg.bf16 and not w16_late and (self.xchg is None or _SHARD_W16_SIDE):
            # (N > 1: beside the row exchange)
            w16_ev = start_w16()
        if self.xchg is not None:
            sparse = {"map": self.map, "slot_row": self.slot_row}
            if lazy and _OWNER_CLAIM_FUSED:
                def owner_claim_catchup(ids, n):
                    # fixed-capacity form: claims + claimed-row catch-up in one launch, the claims
                    # decided by the pre-claim tags the previous step's owner prefetch posted for
                    # this very routing (those with a tag of this step; the rest by CAS)
                    ev = _events(probe, "adam_catchup")
                    pre = self.row_state.view(torch.int64)[:, 0] if (self.prefetch_owner and _OWNER_PF2) else None
                    call("fbn_adam_owner_claim_catchup", ptr(ids), n, int(self.rank == 0), ptr(self.map),
                         ptr(self.slot_row), ptr(pre), ptr(self.E), ptr(self.Em), ptr(self.Ev), self.rows_local, d,
                         self.lazy_window, ptr(self.last), ptr(self.sched), ptr(self.step_dev), self.wd_g,
                         self.beta2, self.eps, *self._pend_args(), int(self.decoupled), st)
                    _events_end(ev)
                    side_pass()
                sparse["claim_catchup"] = owner_claim_catchup
            rows = self.xchg.forward(batch["item_id"], seq, self.E, sparse, self.err,
                                     before_gather=catch_up if lazy else None)
            pos = self.xchg.cur_pos
            fwd_ev = torch.cuda.Event()
            _lib.record_event(fwd_ev, main)
        route_ahead = None
        if self.xchg is not None and next_batch is not None:
            def route_ahead():
                own = self.prefetch_owner and lazy
                self.xchg.prepare(next_batch["item_id"], next_batch.get("item_seq"), self.err, send_rows=own,
                                  after=fwd_ev)
                if own and self.xchg.next_lids is not None:
                    # after this step's claims and window (self.side), once the requests arrived
                    _lib.wait_stream(self.side, self.xchg.side)
                    ev = _events(probe, "adam_prefetch", self.side)
                    call("fbn_adam_prefetch_rows", ptr(self.xchg.next_lids), self.xchg.next_lids.numel(),
                         int(self.rank == 0), self.rows_local, ptr(self.map),
                         ptr(self.row_state.view(torch.int64)[:, 0]) if _OWNER_PF2 else None, ptr(self.E), ptr(self.Em),
                         ptr(self.Ev), d, ptr(self.last), ptr(self.sched), ptr(self.step_dev), self.wd_g, self.beta2,
                         self.eps, *self._pend_args(), int(self.decoupled), self.side.cuda_stream)
                    _events_end(ev, self.side)
                    self.xchg.next_lids.record_stream(self.side)
            if not _ROUTE_AFTER_COMPUTE:
                route_ahead()
                route_ahead = None
        elif self.xchg is None and lazy:
            if w16_late:
                # captured after the claimed-row catch-up's launch, so a graph replay starts the
                # catch-up first; the images follow on the side stream, still beside it (they wait
                # only for what preceded the catch-up)
                step_start = torch.cuda.Event()
                _lib.record_event(step_start, main)
                catch_up(B * (L + 1), claim=True, before_side=step_start)
                w16_ev = self._w16_ev
            else:
                catch_up(B * (L + 1), claim=True, on_side=claim_side)
        elif self.xchg is None:
            call("fbn_claim_rows", ptr(batch["item_id"]), ptr(seq) if L else None, B, L, self.V, ptr(self.map),
                 ptr(self.slot_row), ptr(self.dup), ptr(self.hasdup), st)
        if w16_ev is not None:
            _lib.wait_event(main, w16_ev)
        graphed = False
        # (not inside a graph capture: there each cross-queue edge costs ~10 us of the replay)
        fixup_side = (self.xchg is None and (_FIXUP_ON_SIDE == "1" or (_FIXUP_ON_SIDE == "auto" and not self.side_serial
                                                                        and not torch.cuda.is_current_stream_capturing()))
                      and not self.deterministic and L > 0
                      and not self._early_grad_xchg())
        if (self.xchg is not None and self.shard_graph and probe is None and masks_out is None
                and self.table_adam != "eager" and not self._recording):
            sendbuf = self.xchg.make_sendbuf()
            graphed = self._sharded_compute(batch, labels, pos, cfg, ntot, B, L)
        if not graphed:
            a = ops.forward(self.p, batch, cfg, self.rng, table_rows=rows, pos=pos, err=self.err, labels=labels,
                            w16_ready=w16_ev is not None or w16_main,
                            loss_denom=float(ntot), coll=self.bn_coll, ntot=self._bn_n(ntot, B), acts=self.acts,
                            masks_out=masks_out,
                            probe=probe, count_batches=False,     # num_batches_tracked: fbn_step_end
                            after_gather=start_untouched_adam if self.table_adam == "eager" else None,
                            hooks=side_hooks)
            if self._late_side is not None:
                self._late_side()
                self._late_side = None
            sendbuf = self.xchg.make_sendbuf() if self.xchg is not None else None
            bhooks = {"after_fields_bwd": self._grad_xchg_start} if self._early_grad_xchg() else None
            if fixup_side:
                def fork_fixup():
                    _lib.wait_stream(self.side, main)
                    call("fbn_sparse_fixup_dup", ptr(self.dup), B * (L + 1), ptr(self.gvec), ptr(self.extra),
                         ptr(self.slot_row), L + 1, d, self.side.cuda_stream)
                bhooks = {"after_fields_bwd": fork_fixup}
                if _WGRAD_EARLY and cfg.bf16:
                    def early_wgrad(sums):
                        _lib.wait_stream(self.side, main)
                        sums.launch_group(self.side.cuda_stream, probe, tstream=self.side)
                    bhooks["after_bilinear_bwd"] = early_wgrad
                    bhooks["before_flush"] = lambda: _lib.wait_stream(main, self.side)
            ops.backward(self.p, batch, a, a["gout"], self.g, cfg, gvec=self.gvec if self.xchg is None else None,
                         gnorm=self.gnorm if self.xchg is None else None,
                         pos=pos, sendbuf=sendbuf, coll=self.bn_coll, ntot=self._bn_n(ntot, B),
                         extra_sums=[(a["loss_terms"], B, 1, self.loss, 1.0 / ntot)], probe=probe,
                         hooks=bhooks)
        dense_work = None
        if self.sharded and self._early_grad_xchg() and self.native_comm is None and not self.coll.det:
            # the dense gradients are final once the compute is: their all-reduce goes out now,
            # asynchronously behind the gradient-row all-to-all on the process group's stream,
            # beside the owner's widen / fold / norm; only the loss and the table-gradient sum of
            # squares (known after those) travel at the end
            dense_work = dist.all_reduce(self.flat_g, group=self.coll.group, async_op=True)
        if route_ahead is not None:
            # the host enqueues the next batch's routing (and the owner-side prefetch) only after
            # this step's compute: on the GPU it still starts right after this step's row exchange
            # (it waits on fwd_ev only), but the compute no longer waits for the host to get
            # through ~10 side-stream launches and a collective first
            route_ahead()
        joined = False
        fold_done = False
        if self.xchg is None:
            # single GPU: per-sample vectors; entry e = b*(L+1)+t; duplicates -> extra[claimer]
            n_ent = B * (L + 1)
            if self.deterministic:
                if L == 0:
                    raise ValueError("deterministic mode needs the item_seq history (L > 0)")
                # extra[claimer] becomes the FULL row gradient (Lp1 | FBN_GRAD_FULL for the readers)
                gsrc = (self.gvec, self.extra, (L + 1) | FBN_GRAD_FULL)
                call("fbn_sparse_fold_fx", ptr(self.dup), ptr(self.hasdup), n_ent, ptr(self.gvec), ptr(self.slot_row),
                     gsrc[2], d, ptr(self.fx), st)
            else:
                gsrc = (self.gvec, self.extra, L + 1)
                if fixup_side:
                    _lib.wait_stream(main, self.side)     # the fold (and the side's table passes) done
                    joined = True
                else:
                    call("fbn_sparse_fixup_dup", ptr(self.dup), n_ent, ptr(self.gvec), ptr(self.extra),
                         ptr(self.slot_row), L + 1, d, st)
        else:
            # owner: one received row per entry -- straight into this step's deferred-gradient ring
            # slot when it fits, else a buffer of its own and the rows applied at the step end
            x = self.xchg
            n_ent = x.n_recv
            fold_done = False
            if x.fc_active:
                # fixed-capacity form: the rows arrive in the fixed wire buffer; deferred, they move
                # into ring slot step % ring_n chosen on the device (a replayed step program gets the
                # right slot), and the readers take them through the slot's pointer cell
                wire = x.backward_finish() if x._pending is not None else x.backward(sendbuf)
                defer_now = self.deferred and n_ent <= self.ring_cap
                # (this rank's own block was not sent: its rows are read from the send buffer itself)
                lo, cnt = x.fc_self_rows
                if self._fc_extra is None or self._fc_extra.shape[0] < n_ent:
                    self._fc_extra = _lib.persistent(
                        lambda: torch.zeros((n_ent, d), dtype=torch.float32, device=self.device))
                if defer_now:
                    ring, ring_n, stride = self.ring, self._ring_n_arg(), self._ring_stride()
                else:
                    if self._fc_grad is None or self._fc_grad.shape[0] < n_ent:
                        self._fc_grad = _lib.persistent(
                            lambda: torch.empty((n_ent, d), dtype=torch.float32, device=self.device))
                    ring, ring_n, stride = self._fc_grad, 1, n_ent * d
                rb = FBN_GRAD_BF16 if (defer_now and self.ring_bf16) else 0
                if _OWNER_FOLD or self.deterministic or rb:
                    # the widen into the ring slot and the duplicate fold in one pass: a claimer's row is
                    # stored, a duplicate's added into extra[claimer] (flagged; applied at the tail); the
                    # claimers' squares summed on the way (the flagged ones corrected below).  Deterministic:
                    # the duplicates go to the fixed-point accumulator, extra becomes the FULL row gradient
                    fx = self._fold_bufs(n_ent)
                    call("fbn_owner_fold", ptr(x.recv_ids), n_ent, self.rank, ptr(self.map), ptr(self.slot_row),
                         ptr(wire), int(wire.dtype == torch.bfloat16), ptr(x.fc_send) if cnt else None, lo, cnt,
                         ptr(ring), ring_n, stride, ptr(self.step_dev), ptr(self.ring_cell), ptr(self._fc_extra), d,
                         ptr(self._fc_part), ptr(fx), st)
                    gsrc = (self.ring_cell, self._fc_extra,
                            1 | FBN_GRAD_CELL | rb | (FBN_GRAD_FULL if fx is not None else 0))
                    fold_done = True
                else:
                    call("fbn_ring_slot", ptr(ring), ring_n, stride, ptr(self.step_dev), ptr(self.ring_cell),
                         ptr(wire), int(wire.dtype == torch.bfloat16), n_ent * d, ptr(x.fc_send) if cnt else None,
                         lo * d, cnt * d, st)
                    gsrc = (self.ring_cell, None, 1 | FBN_GRAD_CELL)
            else:
                slot = self._grad_slot()
                defer_now = slot is not None
                if x._pending is not None:          # issued right after the fields backward
                    grows = x.backward_finish()
                else:
                    grows = x.backward(sendbuf, out=slot)
                gsrc = (grows, None, 1)
                g16 = grows.dtype == torch.bfloat16          # received straight into a bf16 ring slot
                if (self.deterministic or g16) and n_ent > 0:
                    # the host-split form (calibration steps, overflow fallbacks): the owner fold in
                    # place over the received rows (the claimer's row is rewritten with itself; ring_n
                    # 1, the cell -> grows) -- deterministic (fixed point), or a bf16 ring slot (no
                    # float atomics into bf16 rows: the duplicates go to extra)
                    fx = self._fold_bufs(n_ent)
                    call("fbn_owner_fold", ptr(x.recv_ids), n_ent, self.rank, ptr(self.map), ptr(self.slot_row),
                         ptr(grows), int(g16), None, 0, 0, ptr(grows), 1 | (FBN_RING_BF16 if g16 else 0), n_ent * d,
                         ptr(self.step_dev), ptr(self.ring_cell), ptr(self._fc_extra), d, ptr(self._fc_part), ptr(fx),
                         st)
                    gsrc = (self.ring_cell, self._fc_extra, 1 | FBN_GRAD_CELL | (FBN_GRAD_BF16 if g16 else 0) |
                            (FBN_GRAD_FULL if fx is not None else 0))
                    fold_done = True
            if not fold_done:
                call("fbn_sparse_fixup", None, None, ptr(x.recv_ids), n_ent, 0, self.V, self.rank, ptr(self.map),
                     ptr(gsrc[0]), None, ptr(self.slot_row), gsrc[2], d, st)
        # clip_grad_norm_(10): dense grads (identical on every rank) + disjoint table shards
        tab_acc = self.sumsq_tab if self.sharded else self.sumsq
        dense_done = False
        if self.xchg is None and L > 0:
            # one process: the dense gradients are final here, so their squares ride along
            fold = not self.sharded and _DENSE_SUMSQ_FOLD
            call("fbn_sumsq_sparse_norms", ptr(self.gnorm), ptr(gsrc[0]), ptr(gsrc[1]), ptr(self.slot_row), gsrc[2],
                 n_ent, d, ptr(tab_acc), ptr(self.fx), ptr(self.flat_g) if fold else None,
                 self.n_dense if fold else 0, st)
            dense_done = fold
        elif fold_done:
            # the fold summed the claimers' own rows; only the flagged ones (duplicates) remain
            call("fbn_sumsq_flagged", ptr(self.slot_row), n_ent, ptr(self.ring_cell), ptr(self._fc_extra), d,
                 ptr(self._fc_part), ptr(tab_acc), ptr(self._fx_sh) if self.deterministic else None,
                 int(bool(gsrc[2] & FBN_GRAD_BF16)), st)
        else:
            call("fbn_sumsq_sparse", ptr(gsrc[0]), ptr(gsrc[1]), ptr(self.slot_row), gsrc[2], n_ent, d, ptr(tab_acc),
                 st)
        if self.sharded:
            # ONE all-reduce: dense grads + the loss + this shard's table-gradient sumsq
            o = self.n_dense
            call("fbn_pack_extras", ptr(self.loss), ptr(self.sumsq_tab), ptr(self.flat_g_ext[o:]), st)
            if dense_work is not None:
                dist.all_reduce(self.flat_g_ext[o:o + 2], group=self.coll.group)
                dense_work.wait()
            else:
                self.coll.allreduce_(self.flat_g_ext[:o + 2])
            if not dense_done:
                # the unpack and the dense gradients' squares in one launch
                call("fbn_unpack_sumsq", ptr(self.flat_g_ext[o:]), ptr(self.loss), ptr(self.flat_g), self.n_dense,
                     ptr(self.sumsq), st)
                dense_done = True
            else:
                call("fbn_unpack_extras", ptr(self.flat_g_ext[o:]), ptr(self.loss), ptr(self.sumsq), st)
        if not dense_done:
            call("fbn_sumsq", ptr(self.flat_g), self.n_dense, None, 0, ptr(self.sumsq), st)
        if not (joined and _JOIN_ONCE):
            # side-stream table pass done before map entries are reset (already joined after the
            # fold: nothing went to the side stream since, and each join costs ~6 us of main-stream idle)
            _lib.wait_stream(main, self.side)
        if self.xchg is None:
            defer_now = self.deferred
        if defer_now:
            # ONE launch: dense Adam with clip_grad_norm_(10), the table step (deferred to each row's
            # next replay; rows with duplicates now), map/slot_row reset, step end
            ev = _events(probe, "adam_tail")
            call("fbn_adam_step_tail", ptr(self.flat_p), ptr(self.flat_g), ptr(self.flat_m), ptr(self.flat_v),
                 self.n_dense, ptr(self.sumsq), self.max_norm, ptr(self.coef), ptr(self.norm), ptr(self.E),
                 ptr(self.Em), ptr(self.Ev), d, ptr(self.map), ptr(gsrc[0]), ptr(gsrc[1]), ptr(self.slot_row), gsrc[2],
                 n_ent, ptr(self.sched), ptr(self.step_dev), self.wd_g, self.beta2, self.eps, ptr(self.last),
                 ptr(self.pend), ptr(self.ring), ptr(self.coef_hist), self._ring_n_arg(), self._ring_stride(), self.B,
                 ptr(self.rng),
                 ptr(self.p["mlp.1.num_batches_tracked"]), ptr(self.p["mlp.5.num_batches_tracked"]), ptr(self.ticket),
                 self.total_steps, ptr(self.err), st)
            _events_end(ev)
        else:
            # clip_grad_norm_(10) is applied inside the dense Adam launch (it publishes coef / norm)
            call("fbn_adam_dense", ptr(self.flat_p), ptr(self.flat_g), ptr(self.flat_m), ptr(self.flat_v),
                 self.n_dense, None, ptr(self.sched), ptr(self.step_dev), self.wd_g, self.beta2, self.eps,
                 ptr(self.sumsq), self.max_norm, ptr(self.coef), ptr(self.norm), st)
            ev = _events(probe, "adam_touched")
            call("fbn_adam_touched", ptr(self.E), ptr(self.Em), ptr(self.Ev), d, ptr(self.map), ptr(gsrc[0]),
                 ptr(gsrc[1]), ptr(self.slot_row), gsrc[2], n_ent, ptr(self.coef), ptr(self.sched),
                 ptr(self.step_dev), self.wd_g, self.beta2, self.eps, ptr(self.last) if lazy else None, st)
            _events_end(ev)
            self.slot_row[:n_ent].fill_(-1)
            call("fbn_step_end", ptr(self.step_dev), ptr(self.rng), ptr(self.sumsq),
                 ptr(self.p["mlp.1.num_batches_tracked"]), ptr(self.p["mlp.5.num_batches_tracked"]), self.total_steps,
                 ptr(self.err), st)
        if self.native_comm is not None:
            # the watchdog's heartbeat (exchange.NativeComm): host time + an event at the step's end;
            # recorded into a step program like any call, so every replay posts it too
            call("fbn_comm_heartbeat", st)
        if self.fc_wanted and not self.xchg.cap and not self.xchg.fc_active:
            self._fc_calibrate()
        self.host_step += 1
        return self.loss

    # ------------------------------------------------------------------ step programs (native step driver)
    def record_program(self, batch: Dict[str, torch.Tensor], labels: torch.Tensor,
                       next_batch: Optional[Dict[str, torch.Tensor]] = None, pool=None,
                       probe: Optional[Dict[str, list]] = None) -> "_lib.StepProgram":
        """Run ONE training step on (batch, labels[, next_batch]) -- a real step, counted -- and record
        it as a step program (csrc/plan.cpp): its ~25 library calls and stream edges, replayed later
        by run_program() with one host call instead of ~0.4 ms of Python per step.

        A replay repeats the recorded step exactly: the same batch tensors (their CURRENT contents
        at replay time), the same next batch for the table-Adam prefetch, the same streams.  Valid
        replays follow the conditions of a hipGraph capture of the step: the step's schedule
        position, dropout stream, claims and deferred gradients are device state (the device step
        counter), nothing host-side changes between replays.  A step that took its row claims from
        the previous step's pre-claims (the next-batch prefetch) replays only after a step that
        prefetched this very batch -- run_program() checks it and raises otherwise; record in the
        order of replay, the step before the first recording given this batch as its next batch.
        One GPU, lazy table Adam with deferred gradients, "all" bilinear (the paths whose step is
        library calls only)."""
        if not (self.table_adam == "lazy" and self.deferred) or self.fcfg.bilinear_each:
            raise ValueError("step programs need the lazy table Adam with deferred gradients and the 'all' "
                             "bilinear interaction")
        seq = batch.get("item_seq")
        key = _batch_key(batch["item_id"], seq if seq is not None and seq.shape[1] else None)
        x = self.xchg
        if x is not None:
            # N > 1: the fixed-capacity exchange over RCCL on the step's stream, this batch routed
            # ahead by the previous step -- then the step is library calls and stream edges only
            if not (x.cap and self.native_comm is not None and next_batch is not None):
                raise ValueError("the sharded step records with the fixed-capacity exchange (after its calibration "
                                 "steps), native RCCL on the step's stream (FBN_NATIVE_COMM=1 at N > 1, or "
                                 "FiBiNETTrainer(native_comm=True); the default at N > 1 is torch.distributed, "
                                 "whose collectives cannot be recorded) and a next batch")
            if x.fc_next is None or x.fc_next[0] != _lib_key(x, batch):
                raise ValueError("record the sharded step after a step that routed this batch ahead (given it as "
                                 "its next_batch)")
        prog = _lib.StepProgram(self.device)
        self._used_pre = False
        self._recording = True
        try:
            with prog.recording(pool):
                # probe (bench): kernel-span probes recorded into the program -- every replay re-arms
                # them, so after a replay each holds that replay's kernel span
                self.step(batch, labels, next_batch=next_batch, probe=probe)
        finally:
            self._recording = False
        if x is not None:
            if not x.fc_active:
                raise RuntimeError("the recorded step's routing overflowed its fixed capacity (it ran with host "
                                   "split sizes): record another step")
            # the routing set this step used, and the next batch's, routed ahead by this step (its
            # event slot: the host waits there for the overflow flag before the next replay)
            prog.fc_cur, prog.fc_after = x.fc_set, x.fc_next
            prog.fc_slot = prog.slot_of(x.fc_next[1]["event"])
            prog.args = (batch, labels, next_batch)
            prog.keep += [x.fc_set, x.fc_next[1]]        # the routing buffers its calls address
        # the claims of the recorded step came from the pre-claims the previous step posted for this
        # very batch (a replay is valid only after such a step), and the step posted its next batch's
        prog.pre_needed, prog.batch_key, prog.pre_key_after = self._used_pre, key, self._pre_key
        prog.batch_ids = (batch["item_id"], seq if seq is not None and seq.shape[1] else None)
        # the tensors the recorded calls address -- the batch, the activation buffers, and every buffer of
        # the trainer's own state as it is NOW: a buffer the trainer later replaces (a fold scratch grown
        # by a larger host-split fallback step) stays alive for this program's replays instead of being
        # freed under its recorded addresses (per-step scratch, zero at rest: the program and the eager
        # steps each keep their own consistent)
        prog.keep += [batch, labels, next_batch, dict(self.acts), [t for _, t in _lib.tensors_of(self)]]
        if _CHECK_POOL:
            self.check_program_memory(prog.pool)
        return prog

    def check_program_memory(self, pool) -> None:
        """Debug check of the step programs' address-lifetime invariant (FBN_CHECK_POOL=1 runs it after
        every record_program): no tensor of the trainer's persistent state -- parameters, moments,
        claims, rings, the exchange's buffers and routing sets, cached scratch and activation buffers --
        lies in the recording pool `pool` (_lib.check_outside_pool)."""
        torch.cuda.synchronize(self.device)
        _lib.check_outside_pool(self, pool)

    def run_program(self, prog: "_lib.StepProgram") -> torch.Tensor:
        """One training step by replaying a recorded step program (see record_program)."""
        if self.host_step >= self.total_steps:
            raise ValueError(f"Tried to step {self.host_step + 1} times. The specified number of total steps is "
                             f"{self.total_steps}")
        if _batch_key(*prog.batch_ids) != prog.batch_key:
            # the ids were rewritten in place since the recording (copy_ bumps the version counter):
            # the pre-claims the previous step posted, and the claims this replay would take from
            # them, are for the old contents -- refuse rather than lose row claims
            raise RuntimeError("step program replayed over batch tensors modified since it was recorded "
                               "(re-record it, or pass fresh tensors to step())")
        x = self.xchg
        if x is not None:
            if x.fc_next is None or x.fc_next[1] is not prog.fc_cur:
                got = "nothing" if x.fc_next is None else (
                    "another batch" if x.fc_next[0] != prog.fc_cur["key"] else "this batch into other buffers")
                raise RuntimeError(f"sharded step program replayed out of order: the previous step routed {got} "
                                   "ahead (record programs in the order they replay, each step given the next batch)")
            if x.fc_overflowed():
                # the routed-ahead ids overflowed a block on some rank (every rank reads the same flag):
                # this step runs eagerly with host-side split sizes, on every rank
                batch, labels, next_batch = prog.args
                return self.step(batch, labels, next_batch=next_batch)
            prog.run()
            x.fc_next = prog.fc_after
            x.fc_wait = lambda: _lib.call_raw("fbn_plan_event_sync", prog.h, prog.fc_slot)
            self.host_step += 1
            return self.loss
        if prog.pre_needed and self._pre_key != prog.batch_key:
            # its recorded claims read pre-claims the previous step did not post for this batch (a
            # replay out of the recorded order): refuse rather than lose row claims
            raise RuntimeError("step program replayed out of order: the previous step did not prefetch its batch "
                               "(record programs in the order they replay, each step given the next batch)")
        prog.run()
        self._pre_key = prog.pre_key_after
        self.host_step += 1
        return self.loss

    def _fc_calibrate(self) -> None:
        """N > 1: after FC_CALIB_STEPS host-split steps, switch the exchange to the fixed-capacity form
        with a per-block capacity of FBN_FC_MARGIN x the largest block seen on any rank (+ 256), capped
        at B * (L + 1) -- a collective, at the same step on every rank."""
        x = self.xchg
        if x.send_counts is not None:
            self._fc_seen = max(self._fc_seen, max(x.send_counts))
        self._fc_steps += 1
        if self._fc_steps < FC_CALIB_STEPS:
            return
        seen = torch.tensor([self._fc_seen], dtype=torch.int64,
                            device="cpu" if self.stage_on_cpu else self.device)
        if dist.is_initialized() and self.world > 1:
            dist.all_reduce(seen, op=dist.ReduceOp.MAX, group=self.group)
        full = self.B * (self.L + 1)
        cap = _FC_CAP if _FC_CAP > 0 else min(full, (int(int(seen.item()) * _FC_MARGIN) + 256 + 63) // 64 * 64)
        self.enable_fixed_exchange(cap)

    def enable_fixed_exchange(self, cap: int) -> None:
        """Exchange in equal-split blocks of cap + 1 slots from the next routed-ahead batch on (the same
        cap on every rank).  Grows the deferred-gradient ring (after bringing every row up to date,
        which clears the pending gradients it holds) and the claim slots when the blocks need more."""
        x = self.xchg
        _lib.persistent(lambda: x.enable_fixed(cap))
        n = x.fc_slots
        if n > self.slot_row.numel():
            self.slot_row = _lib.persistent(lambda: torch.full((n,), -1, dtype=torch.int32, device=self.device))
        if self.deferred and n > self.ring_cap:
            self.flush()
            self.ring_cap = n
            self.ring = _lib.persistent(lambda: self._new_ring((self.ring_n, n, self.d)))
        # the duplicate fold's sums per claimer (zero at rest) and its per-workgroup sums of squares
        # (fbn_owner_fold's 8192-block cap), made here rather than inside a step
        if self._fc_extra is None or self._fc_extra.shape[0] < n:
            self._fc_extra = _lib.persistent(lambda: torch.zeros((n, self.d), dtype=torch.float32, device=self.device))
        if self._fc_part is None:
            self._fc_part = _lib.persistent(lambda: torch.zeros(8192, dtype=torch.float64, device=self.device))
        # the fold's scratch sized for the host-split fallback too (up to every rank's entries at one
        # owner), so a fallback step after recordings never has to grow it
        self._fold_bufs(max(n, self.world * self.B * (self.L + 1)))
        self.fc_wanted = False

    def _fold_bufs(self, n: int):
        """Sharded: the owner fold's buffers for n received slots -- the duplicates' extra rows (zero at
        rest), the per-workgroup partial sums of squares and, in deterministic mode, the fixed-point
        accumulator (returned; None otherwise) -- grown outside any recording pool."""
        d = self.d
        if self.deterministic and (self._fx_sh is None or self._fx_sh.shape[0] < n):
            self._fx_sh = _lib.persistent(lambda: torch.zeros((n, d), dtype=torch.int64, device=self.device))
        if self._fc_extra is None or self._fc_extra.shape[0] < n:
            self._fc_extra = _lib.persistent(lambda: torch.zeros((n, d), dtype=torch.float32, device=self.device))
        if self._fc_part is None:
            self._fc_part = _lib.persistent(lambda: torch.zeros(8192, dtype=torch.float64, device=self.device))
        return self._fx_sh if self.deterministic else None

    def _new_ring(self, shape):
        """The deferred-gradient ring: f32, or (ring_bf16) bf16 with 16 elements of padding past its end
        (the kernels read a bf16 row with the width of an f32 one: csrc/optim.hip ring_load)."""
        if not self.ring_bf16:
            return torch.zeros(shape, dtype=torch.float32, device=self.device)
        n = int(np.prod(shape))
        return torch.zeros(n + 16, dtype=torch.bfloat16, device=self.device)[:n].view(shape)

    def _ring_n_arg(self) -> int:
        """ring_n as the C ABI takes it: | FBN_RING_BF16 for a bf16 ring."""
        return self.ring_n | (FBN_RING_BF16 if self.ring_bf16 else 0)

    def _ring_stride(self) -> int:
        return self.B * 2 * self.d if not self.sharded else self.ring_cap * self.d

    def _sharded_compute(self, batch, labels, pos, cfg, ntot: int, B: int, L: int) -> bool:
        """N > 1: this step's forward + backward (looked-up rows -> per-entry gradient rows in the
        exchange's send buffer) as a replay of the captured segments; False = run it eagerly (the
        first two steps, and once whenever the shapes or the exchange buffers change)."""
        x = self.xchg
        key = (B, L, x.rows_buf.data_ptr(), x.send_buf.data_ptr(),
               tuple((k, tuple(v.shape), v.dtype) for k, v in sorted(batch.items())))
        sg = self._sg
        if sg is None or sg["key"] != key:
            self._sg_eager += 1
            if self._sg_eager <= 2:
                return False
            sg = self._capture(key, batch, labels, pos, cfg, ntot, B)
        pairs = [(v, sg["batch"][k]) for k, v in batch.items()] + [(labels, sg["labels"]), (pos, sg["pos"])]
        _copy_many(pairs, _lib.stream_handle(self.device))
        sg["seg"].replay()
        return True

    def _capture(self, key, batch, labels, pos, cfg, ntot: int, B: int):
        x = self.xchg
        main = torch.cuda.current_stream(self.device)
        sb = {k: v.clone() for k, v in batch.items()}
        sl, sp = labels.clone(), pos.clone()
        self._sg = None
        torch.cuda.synchronize(self.device)
        seg = _Segments(self.coll, torch.cuda.graph_pool_handle())
        bn = seg if self.sync_bn else ops.NO_COLLECTIVE      # local BN: one segment
        cap = torch.cuda.Stream(device=self.device)
        cap.wait_stream(main)
        with torch.cuda.stream(cap):
            seg.begin()
            a = ops.forward(self.p, sb, cfg, self.rng, table_rows=x.rows_buf, pos=sp, err=self.err, labels=sl,
                            loss_denom=float(ntot), coll=bn, ntot=self._bn_n(ntot, B), acts=self.acts,
                            count_batches=False)
            hooks = {"after_fields_bwd": lambda: seg.call(self._grad_xchg_start)} if self._early_grad_xchg() else None
            ops.backward(self.p, sb, a, a["gout"], self.g, cfg, pos=sp, sendbuf=x.send_buf, coll=bn,
                         ntot=self._bn_n(ntot, B), extra_sums=[(a["loss_terms"], B, 1, self.loss, 1.0 / ntot)],
                         hooks=hooks)
            seg.end()
        main.wait_stream(cap)
        # every tensor the segments address stays referenced as long as they live
        self._sg = {"key": key, "seg": seg, "batch": sb, "labels": sl, "pos": sp, "a": a, "acts": dict(self.acts),
                    "bufs": (x.rows_buf, x.send_buf)}
        return self._sg

    def _grad_slot(self):
        """This step's deferred-gradient ring slot, or None (rows applied at once)."""
        if self.deferred and self.xchg.n_recv <= self.ring_cap:
            return self.ring[self.host_step % self.ring_n]
        return None

    def _early_grad_xchg(self) -> bool:
        # the gradient-row all-to-all issued right after the fields backward: native RCCL on the
        # exchange's own stream; torch.distributed asynchronous on its stream (+ the dense all-reduce)
        return self.early_grad_xchg and self.xchg is not None and not self.stage_on_cpu

    def _grad_xchg_start(self) -> None:
        """N > 1: the per-entry gradient rows are complete once the fields backward has run: their
        all-to-all starts there, on the process group's stream, beside the rest of the backward
        (the last parameter reductions and the mm_proj weight gradient)."""
        x = self.xchg
        if x.fc_active:
            x.backward_start(x.fc_send, out=None, early=True)
        else:
            x.backward_start(x.send_buf[:sum(x.send_counts)], out=self._grad_slot(), early=True)

    def _bn_n(self, ntot: int, B: int) -> int:
        """Samples one BatchNorm normalises over: the global batch (SyncBN) or this rank's slice."""
        return ntot if self.sync_bn else B

    def _pend_args(self):
        """(pend, ring, coef_hist, ring_stride, ring_n) of the deferred table gradients (NULLs when off)."""
        if not self.deferred:
            return (None, None, None, 0, 0)
        return (ptr(self.pend), ptr(self.ring), ptr(self.coef_hist), self._ring_stride(), self._ring_n_arg())

    def close(self) -> None:
        """Destroy the native RCCL communicators (the step's and the routing one) and their proxy
        threads; the trainer cannot step at N > 1 afterwards.  Idempotent."""
        if self.xchg is not None and self.xchg.route_comm is not None:
            self.xchg.route_comm.close()
            self.xchg.route_comm = None
        if self.native_comm is not None:
            self.native_comm.close()
            self.native_comm = None
            self.coll.comm = None
            if self.xchg is not None:
                self.xchg.comm = None

    # ------------------------------------------------------------------ inference
    def flush(self) -> None:
        """Bring every table row up to the current step (lazy table Adam); a no-op when eager."""
        if self.table_adam == "lazy":
            call("fbn_adam_flush", ptr(self.E), ptr(self.Em), ptr(self.Ev), self.rows_local, self.d, ptr(self.last),
                 ptr(self.sched), ptr(self.step_dev), self.wd_g, self.beta2, self.eps, *self._pend_args(),
                 int(self.decoupled), _lib.stream_handle(self.device))

    def _bn_from_rank0(self) -> None:
        """Per-rank BatchNorm (sync_bn=False) at N > 1: evaluation uses rank 0's running statistics
        on every rank.  That is nn.DataParallel's behaviour (train_fibinet.py:69-70: each forward
        replicates the module, buffers included, from device 0, and only device 0's updates are
        kept), and they are the statistics the checkpoint holds.  Side effect: the other ranks'
        running statistics are REPLACED by rank 0's (they keep training from those values; only
        rank 0's are ever evaluated or saved).  Broadcast once per evaluation pass: skipped while
        the host step count is unchanged since the last broadcast (4 broadcasts per pass, not per
        batch)."""
        if self.world <= 1 or self.sync_bn:
            return
        if self._bn_synced_at == self.host_step:
            return
        self._bn_synced_at = self.host_step
        for n in ("mlp.1.running_mean", "mlp.1.running_var", "mlp.5.running_mean", "mlp.5.running_var"):
            t = self.p[n]
            if self.stage_on_cpu:
                c = t.cpu()
                dist.broadcast(c, src=0, group=self.group)
                t.copy_(c)
            else:
                dist.broadcast(t, src=0, group=self.group)

    @torch.no_grad()
    def predict(self, batch: Dict[str, torch.Tensor], logits: bool = False) -> torch.Tensor:
        """Eval-mode probabilities (or logits) of this rank's batch.  N > 1: collective (the row
        exchange, and rank 0's BatchNorm statistics when sync_bn is off); a rank with an empty slice
        (a last batch smaller than the world) still joins them and returns an empty tensor."""
        self.flush()
        self._bn_from_rank0()
        cfg = ops.FwdConfig(**{**self.fcfg.__dict__, "training": False})
        cfg.L = batch["item_seq"].shape[1] if "item_seq" in batch else 0
        B = batch["item_id"].shape[0]
        rows = pos = None
        if self.xchg is not None:
            rows = self.xchg.forward(batch["item_id"], batch.get("item_seq"), self.E, {"map": None, "slot_row": None},
                                     self.err)
            pos = self.xchg.cur_pos
        if B == 0:
            return torch.empty(0, dtype=torch.float32, device=self.device)
        a = ops.forward(self.p, batch, cfg, None, table_rows=rows, pos=pos, err=self.err)
        return (a["logits"] if logits else a["probs"]).clone()

    def check_ids(self) -> None:
        """Raise what the reference would have raised since the last check (one 4-byte read):
        IndexError for an id outside its table (nn.Embedding), ValueError for a step past
        total_steps (OneCycleLR) -- the latter is how graph replays, which never pass through
        step()'s host-side guard, report it (the device step counter saturates)."""
        e = int(self.err.item())
        if e & 1:
            raise IndexError("index out of range in self (item/likes/views id outside its embedding table)")
        if e & 2:
            raise ValueError(f"Tried to step more than {self.total_steps} times. The specified number of total steps "
                             f"is {self.total_steps}")

    def device_step(self) -> int:
        """Optimizer steps taken (the device counter: also advanced by hipGraph replays)."""
        return int(self.step_dev.item())

    def current_lr(self) -> float:
        return self.lrs[min(self.device_step(), self.total_steps - 1)]

    # ------------------------------------------------------------------ checkpoint (App. B keys)
    def state_dict(self, all_ranks: bool = False) -> Dict[str, torch.Tensor]:
        """Reference state_dict (App. B keys, CPU tensors).  N > 1: collective; the full table is
        assembled on rank 0 only (the rank that saves the checkpoint, train_fibinet.py:148-152) --
        every other rank gets the same dict without ``item_emb.weight`` -- unless all_ranks.  The
        shards travel to rank 0 in chunks of <= 256 MB through one device staging buffer, straight
        into one host tensor, so a C5 shard (12.5 M rows x 128, 6.4 GB) never needs a second full
        copy on any GPU."""
        self.flush()
        out = {}
        if self.world > 1:
            full = self._gather_table(all_ranks)
        else:
            full = self.E.detach().cpu().clone()
        for k in self.key_order:
            if k == TABLE:
                if full is not None:
                    out[k] = full
            else:
                out[k] = self.p[k].detach().cpu().clone()
        return out

    _loaded_table = None

    def _scatter_table(self, full: Optional[torch.Tensor]) -> None:
        """Rank 0's full table -> every rank's row block (the inverse of _gather_table; chunks of
        <= 256 MB through one staging buffer)."""
        if self.rank == 0 and full is None:
            raise KeyError(f"load_state_dict at N > 1: rank 0's dict must hold {TABLE!r} (state_dict() "
                           f"gives it to rank 0; state_dict(all_ranks=True) to every rank)")
        d, Vl = self.d, self.Vl
        chunk = max(1, (256 << 20) // (d * 4))
        dev = "cpu" if self.stage_on_cpu else self.device
        stage = torch.empty((min(chunk, Vl), d), dtype=torch.float32, device=dev)
        for dst in range(self.world):
            lo = dst * Vl
            n = max(0, min(self.V, lo + Vl) - lo)
            for c0 in range(0, n, chunk):
                c1 = min(n, c0 + chunk)
                buf = stage[:c1 - c0]
                if self.rank == 0:
                    buf.copy_(full[lo + c0:lo + c1])
                if dst != 0:
                    if self.rank == 0:
                        dist.send(buf, dst=dst, group=self.group)
                    elif self.rank == dst:
                        dist.recv(buf, src=0, group=self.group)
                if self.rank == dst:
                    self.E[c0:c1].copy_(buf)
        self._loaded_table = True

    def _gather_table(self, all_ranks: bool) -> Optional[torch.Tensor]:
        d, Vl = self.d, self.Vl
        chunk = max(1, (256 << 20) // (d * 4))
        dev = "cpu" if self.stage_on_cpu else self.device
        me = all_ranks or self.rank == 0
        full = torch.empty((self.V, d), dtype=torch.float32) if me else None
        stage = torch.empty((min(chunk, Vl), d), dtype=torch.float32, device=dev)
        for src in range(self.world):
            lo = src * Vl
            n = max(0, min(self.V, lo + Vl) - lo)
            for c0 in range(0, n, chunk):
                c1 = min(n, c0 + chunk)
                buf = stage[:c1 - c0]
                if src == self.rank:
                    buf.copy_(self.E[c0:c1])
                if all_ranks:
                    dist.broadcast(buf, src=src, group=self.group)
                elif src != 0:
                    if self.rank == src:
                        dist.send(buf, dst=0, group=self.group)
                    elif self.rank == 0:
                        dist.recv(buf, src=src, group=self.group)
                if me:
                    full[lo + c0:lo + c1].copy_(buf)
        return full

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        """Load reference-format weights (App. B keys).  Like ``model.load_state_dict`` under the
        reference's loop, the optimizer state (Adam moments, step count, schedule position) is kept:
        only the weights and BatchNorm buffers change.

        N > 1: collective when any rank's dict lacks ``item_emb.weight`` -- the form state_dict()
        returns on ranks above 0 -- so ``load_state_dict(state_dict())`` round-trips on every rank:
        rank 0 (which must hold the table) sends each rank its row block; ranks whose dict holds the
        full table take their block from it."""
        self.flush()
        if self.world > 1:
            # [ranks holding the table, rank 0 holds it]: every rank decides (and raises) together --
            # a rank-0-only KeyError would leave the others blocked in _scatter_table's recv
            have = torch.tensor([int(TABLE in sd), int(self.rank == 0 and TABLE in sd)], dtype=torch.int32,
                                device="cpu" if self.stage_on_cpu else self.device)
            dist.all_reduce(have, group=self.group)
            n_have, rank0_has = (int(x) for x in have.tolist())
            if n_have < self.world:
                if not rank0_has:
                    raise KeyError(f"load_state_dict at N > 1: rank 0's dict must hold {TABLE!r} (state_dict() "
                                   f"gives it to rank 0; state_dict(all_ranks=True) to every rank)")
                self._scatter_table(sd.get(TABLE) if self.rank == 0 else None)
        for k in self.key_order:
            if k == TABLE:
                if self.world == 1 or TABLE in sd and self._loaded_table is None:
                    self.E.copy_(sd[k][self.rows_lo:self.rows_lo + self.rows_local].to(self.device))
                self._loaded_table = None
            else:
                self.p[k].copy_(sd[k].to(self.device))
        self.last.copy_(self.step_dev.expand_as(self.last))     # loaded rows are current (device step)
        if self.pend is not None:
            self.pend.fill_(-1)
