"""Row-sharded item table exchange over torch.distributed (RCCL on MI355X, gloo in CPU tests).

One process per GPU.  The item table E (V x d) is split into contiguous row blocks of
``Vl = ceil(V / world)`` rows (owner = id // Vl).  Replaces the reference's
``torch.nn.DataParallel`` (src/train_fibinet.py:69-70), which broadcast the whole table to
every GPU and reduced its dense gradient back every step.

Forward  (requester -> owner -> requester):
  route (ids -> per-owner int32 local rows + pos[b][t])  ->  all_to_all(counts)  ->
  all_to_all(ids)  ->  owner gather (+ register rows for the sparse gradient)  ->
  all_to_all(rows)  ->  fields_fwd reads rows[pos]
Backward (the sparse reduce-scatter):
  fields_bwd writes one gradient row per routed entry  ->  all_to_all(rows)  ->  the received
  rows are the owner's sparse gradient (slot = received entry; fbn_sparse_fixup folds rows hit
  by several entries into the entry that claimed the row in the forward).
Split sizes need a host read of the N routed counts per step (all_to_all_single takes host
split lists).  ``prepare(next_batch)`` takes that read and the ids all-to-all off the critical
path: the next batch is routed on a side stream while the current step runs and sent to the
owners as ONE equal-split all-to-all of padded per-owner blocks that carry their counts; the
owners pack the ids on device and both count vectors land in pinned host memory -- the next
forward starts at the owner's claims with no collective before them (two routing buffer sets
alternate).  Without it the forward routes inline: a counts all-to-all, one host sync, an ids
all-to-all.

Fixed-capacity form (enable_fixed(cap), the trainer's default once calibrated): requester r's
block for owner o has cap + 1 slots, so the ids, the looked-up rows and the gradient rows all cross
as EQUAL-split all-to-alls and no split size reaches the host; the owner works on the
world * (cap + 1) slots as they arrive (negative id = empty slot) and a step is a fixed sequence
of library calls -- recordable as a step program (trainer.record_program).  An entry past a block's
capacity is not routed; the overflow travels in-band with the ids (every block's last slot), so
every rank reads the same global flag before the step and all of them exchange that step with
host-side split sizes instead (fbn_route_fc / fbn_route_fc_status).
"""
from __future__ import annotations

import ctypes
import os
import sys
import time
from typing import Optional

import torch
import torch.distributed as dist

from . import _lib
from ._lib import call, ptr


def _torch_rccl() -> str:
    """The RCCL library torch's process groups use (torch/lib/librccl.so), so the native
    communicators share its runtime; the system one if torch carries none."""
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else "librccl.so.1"


_DEBUG_FC = os.environ.get("FBN_DEBUG_FC") == "1"     # diagnostics: trace the fixed-capacity routing
_DTYPE_CODE = {torch.float32: 0, torch.float64: 1, torch.int32: 2}


class NativeComm:
    """An RCCL communicator driven through the C-ABI (csrc/comm.cpp): collectives enqueued on the
    CALLER's stream, between the step's kernels, with no cross-queue edges (torch.distributed runs
    each collective on its process group's own stream behind two event edges, ~10-20 us apiece).
    Creation is collective over `group` (rank 0's unique id is broadcast through it)."""

    def __init__(self, world: int, rank: int, group=None, device=None):
        call("fbn_comm_load", _torch_rccl().encode())
        n = _lib.lib().fbn_comm_id_bytes()
        uid = (ctypes.c_char * n)()
        if rank == 0:
            call("fbn_comm_unique_id", uid)
        obj = [bytes(uid) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0 if group is None else dist.get_global_rank(group, 0), group=group)
        uid = (ctypes.c_char * n).from_buffer_copy(obj[0])
        h = ctypes.c_void_p()
        with torch.cuda.device(device if device is not None else torch.cuda.current_device()):
            call("fbn_comm_init", ctypes.byref(h), uid, world, rank)
            if COMM_TIMEOUT_S > 0:
                # the step's heartbeats (trainer: fbn_comm_heartbeat at every step's end) feed it
                call("fbn_comm_watch", int(COMM_TIMEOUT_S * 1000))
        self.handle, self.world, self.rank = h.value, world, rank

    @staticmethod
    def watchdog_fired() -> bool:
        """The watchdog aborted the communicators (no step completed within FBN_COMM_TIMEOUT_S)."""
        return bool(_lib.lib().fbn_comm_watchdog_fired(None))

    def alltoallv(self, out: torch.Tensor, inp: torch.Tensor, recv_counts, send_counts) -> None:
        """Rows (dim 0) of inp to the ranks, send_counts[r] to rank r; recv_counts[r] rows from r."""
        row_bytes = inp.element_size()
        for n in inp.shape[1:]:          # (an empty inp -- a rank asked for no rows -- has shape (0, d))
            row_bytes *= n
        sc = (ctypes.c_int * self.world)(*send_counts)
        rc = (ctypes.c_int * self.world)(*recv_counts)
        call("fbn_comm_alltoallv", self.handle, ptr(inp), sc, ptr(out), rc, row_bytes,
             _lib.stream_handle(out.device))

    def alltoall(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        """Equal split: inp.numel() / world elements to every rank."""
        call("fbn_comm_alltoall", self.handle, ptr(inp), ptr(out), inp.numel() * inp.element_size() // self.world,
             _lib.stream_handle(out.device))

    def alltoall_peers(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        """Equal split without this rank's own block (it stays where it is; nothing at one rank)."""
        call("fbn_comm_alltoall_peers", self.handle, ptr(inp), ptr(out),
             inp.numel() * inp.element_size() // self.world, _lib.stream_handle(out.device))

    def allreduce_(self, t: torch.Tensor) -> None:
        call("fbn_comm_allreduce", self.handle, ptr(t), t.numel(), _DTYPE_CODE[t.dtype], _lib.stream_handle(t.device))

    def allgather(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        """out [world * n] <- every rank's inp [n], in rank order."""
        call("fbn_comm_allgather", self.handle, ptr(inp), ptr(out), inp.numel() * inp.element_size(),
             _lib.stream_handle(out.device))

    def close(self) -> None:
        if self.handle:
            call("fbn_comm_destroy", self.handle)
            self.handle = None


def native_comm_wanted(device, group=None, stage_on_cpu: bool = False, force: Optional[bool] = None) -> bool:
    """RCCL on the step's stream: a HIP device and an nccl (= RCCL) process group.  FBN_NATIVE_COMM
    = 1: always; 0: never (torch.distributed's collectives, on its own stream); "auto" (default): at
    world = 1 only (the sharded smoke job, where it is tested against the torch.distributed path).
    At world > 1 the native communicators have never run on hardware (RCCL refuses two ranks on
    one device, and no multi-GPU box was available), and they bypass torch's watchdog timeouts, so
    the default keeps torch.distributed's collectives there until a multi-GPU run shows loss and
    table parity between the two."""
    mode = os.environ.get("FBN_NATIVE_COMM", "auto") if force is None else ("1" if force else "0")
    if not (torch.device(device).type == "cuda" and not stage_on_cpu and dist.is_initialized()
            and dist.get_backend(group) == "nccl") or mode == "0":
        return False
    return mode == "1" or dist.get_world_size(group) == 1


# the native communicators' watchdog (csrc/comm.cpp): abort them all when no step has completed for
# this many seconds (torch.distributed's process groups have their own collective timeout; these
# communicators bypass it).  0 disables it.
COMM_TIMEOUT_S = float(os.environ.get("FBN_COMM_TIMEOUT_S", "300"))


class HipExchangeKernels:
    """Device kernels of the exchange (exchange.hip)."""

    def pad_routes(self, send_ids, offsets, counts, world, cap, out):
        call("fbn_pad_routes", ptr(send_ids), ptr(offsets), ptr(counts), world, cap, ptr(out),
             _lib.stream_handle(out.device))

    def route(self, item, seq, B, L, V, Vl, world, counts, offsets, cursor, send_ids, pos, err):
        call("fbn_route", ptr(item), ptr(seq), B, L, V, Vl, world, ptr(counts), ptr(offsets), ptr(cursor),
             ptr(send_ids), ptr(pos), ptr(err), _lib.stream_handle(item.device))

    def owner_claim(self, ids, map_, slot_row, rank):
        call("fbn_owner_claim", ptr(ids), ids.shape[0], ptr(map_), ptr(slot_row), rank, _lib.stream_handle(ids.device))

    def owner_gather(self, ids, E, out, map_, slot_row, rank, d):
        call("fbn_owner_gather", ptr(ids), ids.shape[0], ptr(E), ptr(out), ptr(map_), ptr(slot_row), rank, d,
             int(out.dtype == torch.bfloat16),
             _lib.stream_handle(E.device))

    def compact_routes(self, padded, world, cap, ids, counts):
        call("fbn_compact_routes", ptr(padded), world, cap, ptr(ids), ptr(counts), _lib.stream_handle(ids.device))

    def widen(self, inp, out):
        call("fbn_widen_bf16", ptr(inp), ptr(out), inp.numel(), _lib.stream_handle(out.device))

    def route_fc(self, item, seq, B, L, V, Vl, world, cap, send_ids, pos, stat, err):
        call("fbn_route_fc", ptr(item), ptr(seq), B, L, V, Vl, world, cap, ptr(send_ids), ptr(pos), ptr(stat), ptr(err),
             _lib.stream_handle(item.device))

    def route_fc_status(self, send_ids, recv_ids, world, rank, cap, stat, host):
        call("fbn_route_fc_status", ptr(send_ids), ptr(recv_ids), world, rank, cap, ptr(stat), ptr(host),
             _lib.stream_handle(recv_ids.device))

    def owner_gather_self(self, ids, E, out, map_, slot_row, rank, d, self_out, self_lo, self_n):
        call("fbn_owner_gather_self", ptr(ids), ids.shape[0], ptr(E), ptr(out), ptr(map_), ptr(slot_row), rank, d,
             int(out.dtype == torch.bfloat16), ptr(self_out), self_lo, self_n, _lib.stream_handle(E.device))


def _pad4(n: int) -> int:
    return (n + 3) // 4 * 4


# fixed-capacity routing sets kept, one per distinct batch (~2 MB of device memory each at C3, and a
# pinned host word block): at most FC_SET_BYTES of them (FBN_FC_SET_BYTES, default 1 GiB; at least 8
# sets), the oldest forgotten first.  A step program holds the sets its calls address (prog.keep), so
# forgetting one never frees memory a program still uses; a forgotten batch is routed into a new set
# the next time it comes round.
FC_SET_BYTES = int(os.environ.get("FBN_FC_SET_BYTES", str(1 << 30)))


class RowExchange:
    def __init__(self, rank: int, world: int, V: int, d: int, B: int, L: int, device, group=None, kernels=None,
                 stage_on_cpu: bool = False, rows_bf16: bool = False, side=None, comm: Optional[NativeComm] = None):
        self.rank, self.world, self.V, self.d, self.L, self.B = rank, world, V, d, L, B
        self.Vl = (V + world - 1) // world
        self.group = group
        self.k = kernels or HipExchangeKernels()
        self.device = device
        self.stage_on_cpu = stage_on_cpu          # gloo on a GPU box: collectives on host copies
        self.comm = comm                          # RCCL on the caller's stream (NativeComm) or None
        self.route_comm = None
        # bf16 mode: looked-up rows AND per-entry gradient rows cross the wire as bf16 (half the
        # bytes of both all-to-alls; the fields kernel widens the rows on load, the owner widens the
        # gradient rows on receipt and folds them in f32)
        self.row_dtype = torch.bfloat16 if rows_bf16 else torch.float32
        i32 = dict(dtype=torch.int32, device=device)
        # two routing buffer sets: the step in flight uses one while prepare() fills the other
        self.sets = []
        for _ in range(2):
            self.sets.append({"counts": torch.zeros(world, **i32), "offsets": torch.zeros(world + 1, **i32),
                              "cursor": torch.zeros(world, **i32), "send_ids": torch.empty(B * (L + 1), **i32),
                              "pos": torch.empty((B, L + 1), **i32), "recv_counts": torch.zeros(world, **i32),
                              "recv_ids": None,
                              "host": torch.zeros(2 * world, dtype=torch.int32,
                                                  pin_memory=torch.device(device).type == "cuda"),
                              "event": None, "key": None})
        self.cur = 0
        self.side = None
        self.route_group = group
        if torch.device(device).type == "cuda" and dist.is_initialized():
            # the caller's side stream when given (the trainer's: a process has 4 hardware queues,
            # GPU_MAX_HW_QUEUES, and a stream of its own here landed on the main stream's queue,
            # serialising the next batch's routing with this step's compute)
            self.side = side if side is not None else torch.cuda.Stream(device=device)
            # a communicator of its own: the next batch's counts exchange runs beside this step's
            # collectives instead of queueing between them (every rank creates it here, in order)
            if comm is not None:
                self.route_comm = NativeComm(world, rank, group, device)
            else:
                self.route_group = dist.new_group(ranks=list(range(world)))
        self.send_counts = None
        self.recv_counts = None
        self.recv_ids = None
        self.next_lids = None
        self.host_wait_s = 0.0      # host time blocked on the routed-ahead counts (bench diagnostics)
        # looked-up rows and per-entry gradient rows live in buffers that only grow (each step uses a
        # prefix): fixed addresses, so the trainer's compute between the exchanges can be a hipGraph
        self.rows_buf = None
        self.send_buf = None
        self._pending = None        # gradient-row all-to-all issued by backward_start()
        self._comm_stream = None    # native RCCL, early gradient exchange: its stream
        # fixed-capacity form (enable_fixed): slots per requester -> owner block, 0 = off
        self.cap = 0
        self.fc_sets = {}           # batch key -> its routing buffers (kept: step programs address them)
        self.fc_next = None         # (key, set): the next batch, routed ahead in the fixed-capacity form
        self.fc_wait = None         # host wait for that routing (an event, or a step program's event slot)
        self.fc_active = False      # this step exchanges in the fixed-capacity form
        self.fc_set = None          # ... and this is its routing set
        self.fc_fallbacks = 0       # steps exchanged with host split sizes after an overflow

    # ------------------------------------------------------------------ fixed-capacity form
    def enable_fixed(self, cap: int) -> None:
        """Exchange in equal-split blocks of cap + 1 slots per (requester, owner) pair from the next
        routed-ahead batch on (cap must be the same on every rank)."""
        self.cap = int(cap)
        n = self.fc_slots
        self.fc_rows = torch.empty((n, self.d), dtype=self.row_dtype, device=self.device)    # requester: rows[pos]
        self.fc_reply = torch.empty((n, self.d), dtype=self.row_dtype, device=self.device)   # owner: gathered rows
        self.fc_send = torch.empty((n, self.d), dtype=self.row_dtype, device=self.device)    # requester: grad rows
        self.fc_wire = torch.empty((n, self.d), dtype=self.row_dtype, device=self.device)    # owner: received grads
        self.fc_sets = {}
        self.fc_next = None
        # native RCCL: this rank's own block never crosses the all-to-alls (fbn_comm_alltoall_peers) --
        # the owner writes its looked-up rows straight into the requester's row buffer and reads the
        # requester's gradient rows from its send buffer
        self.fc_self = self.comm is not None

    @property
    def fc_slots(self) -> int:
        return self.world * (self.cap + 1)

    @property
    def fc_self_rows(self):
        """(first row, rows) of this rank's own block when it stays in place, else (0, 0)."""
        return (self.rank * (self.cap + 1), self.cap + 1) if self.fc_self else (0, 0)

    def _a2a_fc(self, out, inp, route=False):
        """Equal-split all-to-all of the fixed-capacity form (own block skipped when it stays in place)."""
        if self.fc_self:
            (self.route_comm if route else self.comm).alltoall_peers(out, inp)
        else:
            self._a2a(out, inp, None, None, self.route_group if route else None, route=route)

    def _fc_routing_set(self, key):
        st = self.fc_sets.get(key)
        if st is None:
            n = self.fc_slots
            per_set = 4 * (2 * n + self.B * (self.L + 1) + 2 * _pad4(self.world + 1))
            if len(self.fc_sets) >= max(8, FC_SET_BYTES // per_set):   # forget the oldest (a program holds its own)
                self.fc_sets.pop(next(iter(self.fc_sets)))
            i32 = dict(dtype=torch.int32, device=self.device)
            # (a set outlives the step that routes into it: never from a program's recording pool)
            st = _lib.persistent(lambda: {
                "send_ids": torch.empty(n, **i32), "recv_ids": torch.empty(n, **i32),
                "pos": torch.empty((self.B, self.L + 1), **i32), "stat": torch.zeros(_pad4(self.world + 1), **i32),
                "host": torch.zeros(_pad4(self.world + 1), dtype=torch.int32,
                                    pin_memory=torch.device(self.device).type == "cuda"),
                "event": None, "key": key})
            self.fc_sets[key] = st
        return st

    def _prepare_fc(self, item, seq, err, send_rows, after) -> None:
        """prepare() in the fixed-capacity form: route, the ids all-to-all (equal split) and the
        global overflow flag, all on the side stream with no host involvement; the flag lands in
        pinned memory for the next forward's host check."""
        B = item.shape[0]
        L = 0 if seq is None else seq.shape[1]
        key = self._key(item, seq)
        if self.side is None:
            st = self._fc_routing_set(key)
        else:
            # allocated on the side stream, which writes it while the main stream is still running
            # this step's backward: a block the main stream freed earlier in the step (still in use
            # by its queued kernels -- and by a step program's replays, at the recorded addresses)
            # must not come back here
            with torch.cuda.stream(self.side):
                st = self._fc_routing_set(key)
        if self.side is None:
            # CPU ranks (gloo tests): routed inline, nothing to wait for
            self.k.route_fc(item, seq if L else None, B, L, self.V, self.Vl, self.world, self.cap, st["send_ids"],
                            st["pos"], st["stat"], err)
            self._a2a_fc(st["recv_ids"], st["send_ids"], route=True)
            self.k.route_fc_status(st["send_ids"] if self.fc_self else None, st["recv_ids"], self.world, self.rank,
                                   self.cap, st["stat"], st["host"])
            self.fc_next, self.fc_wait = (key, st), (lambda: None)
            if send_rows:
                self.next_lids = st["recv_ids"]
            return
        main = torch.cuda.current_stream(item.device)
        if after is None:
            _lib.wait_stream(self.side, main)
        else:
            _lib.wait_event(self.side, after)
        with torch.cuda.stream(self.side):
            self.k.route_fc(item, seq if L else None, B, L, self.V, self.Vl, self.world, self.cap, st["send_ids"],
                            st["pos"], st["stat"], err)
            self._a2a_fc(st["recv_ids"], st["send_ids"], route=True)
            self.k.route_fc_status(st["send_ids"] if self.fc_self else None, st["recv_ids"], self.world, self.rank,
                                   self.cap, st["stat"], st["host"])
        ev = torch.cuda.Event()
        _lib.record_event(ev, self.side)
        st["event"] = ev
        self.fc_next = (key, st)
        self.fc_wait = ev.synchronize
        if send_rows:
            self.next_lids = st["recv_ids"]
        if _DEBUG_FC:
            print(f"[fc] prepare key {key[0] % 100000} set {id(st) % 100000}", file=sys.stderr, flush=True)

    def fc_overflowed(self) -> bool:
        """Host: wait for the routed-ahead batch's routing and read its global overflow flag (the
        same value on every rank)."""
        t0 = time.perf_counter()
        self.fc_wait()
        self.host_wait_s += time.perf_counter() - t0
        return int(self.fc_next[1]["host"][0]) != 0

    def _forward_fc(self, st, E_local, sparse, err, before_gather) -> torch.Tensor:
        self.fc_active, self.fc_set = True, st
        self.cur_pos = st["pos"]
        self.recv_ids = st["recv_ids"]
        self.send_counts = self.recv_counts = None
        n = self.fc_slots
        claim = before_gather is not None and sparse.get("map") is not None
        if claim and sparse.get("claim_catchup") is not None:
            # the claims and the claimed-row catch-up in one launch (the trainer's lazy table Adam)
            sparse["claim_catchup"](self.recv_ids, n)
        elif claim:
            self.k.owner_claim(self.recv_ids, sparse["map"], sparse["slot_row"], self.rank)
            before_gather(n)
        m, sr = (None, None) if claim else (sparse["map"], sparse["slot_row"])
        if self.fc_self:
            lo, cnt = self.fc_self_rows
            self.k.owner_gather_self(self.recv_ids, E_local, self.fc_reply, m, sr, self.rank, self.d, self.fc_rows,
                                     lo, cnt)
        else:
            self.k.owner_gather(self.recv_ids, E_local, self.fc_reply, m, sr, self.rank, self.d)
        self._a2a_fc(self.fc_rows, self.fc_reply)
        self.rows_buf = self.fc_rows
        return self.fc_rows

    @property
    def n_recv(self) -> int:
        """Owner-side entries of this step (received slots, empty ones included in the fixed form)."""
        return self.fc_slots if self.fc_active else sum(self.recv_counts)

    @property
    def n_send(self) -> int:
        return self.fc_slots if self.fc_active else sum(self.send_counts)

    @property
    def rows_lo(self) -> int:
        return self.rank * self.Vl

    @property
    def rows_local(self) -> int:
        return max(0, min(self.V, (self.rank + 1) * self.Vl) - self.rows_lo)

    def _a2a(self, out, inp, out_splits, in_splits, group=None, route=False):
        """out <- all-to-all of inp (rows; splits None = equal) on the current stream."""
        if self.comm is not None:
            comm = self.route_comm if route else self.comm
            if out_splits is None:
                comm.alltoall(out, inp)
            else:
                comm.alltoallv(out, inp, out_splits, in_splits)
            return out
        group = group if group is not None else self.group
        if not self.stage_on_cpu:
            dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)
            return out
        o = out.cpu()
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
        return out

    @property
    def pos(self):
        return self.sets[self.cur]["pos"]

    def _route(self, st, item, seq, err, group=None, exchange_counts=True):
        B = item.shape[0]
        L = 0 if seq is None else seq.shape[1]
        if L != self.L:
            st["pos"] = torch.empty((B, L + 1), dtype=torch.int32, device=item.device)
        pos = st["pos"][:B, :L + 1]
        self.k.route(item, seq, B, L, self.V, self.Vl, self.world, st["counts"], st["offsets"], st["cursor"],
                     st["send_ids"], pos, err)
        if exchange_counts:
            self._a2a(st["recv_counts"], st["counts"], None, None, group)
        return pos

    @staticmethod
    def _key(item, seq):
        # the prepared routing is used only for the very tensors it was computed from, unmodified
        # since (a copy_ into the same buffer bumps the version counter)
        return (item.data_ptr(), item.shape[0], item._version, 0 if seq is None else seq.data_ptr(),
                0 if seq is None else seq.shape[1], 0 if seq is None else seq._version)

    def prepare(self, item, seq, err, send_rows: bool = False, after=None) -> None:
        """Route the NEXT step's batch now, on a side stream (HIP device only), and deliver it to the
        owners as ONE equal-split all-to-all of the padded routing (fbn_pad_routes: each
        destination's ids padded to cap, its count in the last slot): the owner recovers the counts
        and the packed ids on device (fbn_compact_routes), and both count vectors land in pinned
        host memory -- the next forward reads them without a sync on the main stream and runs no
        counts / ids all-to-all.  Used by the next forward() only if it gets the same
        id tensors, unmodified (address, shape and version counter); otherwise that forward routes
        inline.  send_rows: also expose the
        received padded blocks as self.next_lids [world * (cap + 1)] (negative = no row), ready on
        self.side -- the owner's table-Adam prefetch (fbn_adam_prefetch_rows) reads them."""
        self.next_lids = None
        if self.cap and item.shape[0] == self.B and (0 if seq is None else seq.shape[1]) == self.L:
            self._prepare_fc(item, seq, err, send_rows, after)
            return
        if self.side is None:
            return
        st = self.sets[1 - self.cur]
        main = torch.cuda.current_stream(item.device)
        # the ids and the buffer set are free: after everything on the main stream so far, or after
        # `after` (an event the caller recorded once this step's row exchange was enqueued)
        if after is None:
            self.side.wait_stream(main)
        else:
            self.side.wait_event(after)
        B = item.shape[0]
        cap = B * (1 + (0 if seq is None else seq.shape[1]))
        with torch.cuda.stream(self.side):
            st["pos_view"] = self._route(st, item, seq, err, exchange_counts=False)
            padded = torch.empty(self.world * (cap + 1), dtype=torch.int32, device=item.device)
            self.k.pad_routes(st["send_ids"], st["offsets"], st["counts"], self.world, cap, padded)
            recv = torch.empty_like(padded)
            self._a2a(recv, padded, None, None, self.route_group, route=True)
            if st["recv_ids"] is None or st["recv_ids"].numel() < self.world * cap:
                st["recv_ids"] = torch.empty(self.world * cap, dtype=torch.int32, device=item.device)
            self.k.compact_routes(recv, self.world, cap, st["recv_ids"], st["recv_counts"])
            st["host"][:self.world].copy_(st["counts"], non_blocking=True)
            st["host"][self.world:].copy_(st["recv_counts"], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.side)
            if send_rows:
                self.next_lids = recv
        for t in (item, seq, err):
            if t is not None:
                t.record_stream(self.side)
        st["event"], st["key"] = ev, self._key(item, seq)

    def forward(self, item, seq, E_local, sparse, err, before_gather=None) -> torch.Tensor:
        """Returns the requester's row buffer [n_sent, d]; self.pos maps (b, t) -> row (or -1).
        before_gather(n_recv): runs at the owner between registering the requested rows in the
        sparse map and gathering them (the lazy table Adam brings them up to date there)."""
        B = item.shape[0]
        L = 0 if seq is None else seq.shape[1]
        self.fc_active = False
        if _DEBUG_FC:
            print(f"[fc] forward key {self._key(item, seq)[0] % 100000} next "
                  f"{None if self.fc_next is None else (self.fc_next[0][0] % 100000, id(self.fc_next[1]) % 100000)}",
                  file=sys.stderr, flush=True)
        if self.fc_next is not None and self.fc_next[0] == self._key(item, seq):
            st = self.fc_next[1]
            if not self.fc_overflowed():
                self.fc_next = None
                if not _lib.recording() and item.device.type == "cuda":
                    # (a recorded step relies on the previous step's closing join of the side stream)
                    _lib.wait_event(torch.cuda.current_stream(item.device), st["event"])
                return self._forward_fc(st, E_local, sparse, err, before_gather)
            self.fc_fallbacks += 1                    # every rank read the same flag: all route inline
        self.fc_next = None
        nxt = self.sets[1 - self.cur]
        if nxt["event"] is not None and nxt["key"] == self._key(item, seq):
            # routed ahead by prepare(): wait for the side stream's copy only, then order the
            # main stream after the side stream's routing work
            self.cur = 1 - self.cur
            st = self.sets[self.cur]
            t0 = time.perf_counter()
            st["event"].synchronize()
            self.host_wait_s += time.perf_counter() - t0
            torch.cuda.current_stream(item.device).wait_event(st["event"])
            st["event"] = None
            h = st["host"].tolist()
            sc, rc = h[:self.world], h[self.world:]
            pos = st["pos_view"]
            prepared = True
        else:
            if nxt["event"] is not None:              # prepared for other tensors: drop it
                nxt["event"].synchronize()
                nxt["event"] = None
            st = self.sets[self.cur]
            pos = self._route(st, item, seq, err)
            sc = st["counts"].tolist()
            rc = st["recv_counts"].tolist()       # the one host sync of the step
            prepared = False
        self.cur_pos = pos.contiguous()
        self.send_counts, self.recv_counts = sc, rc
        n_send, n_recv = sum(sc), sum(rc)
        if prepared:          # the requests arrived with the routing (prepare): packed on the owner
            self.recv_ids = st["recv_ids"][:n_recv]
        else:
            self.recv_ids = torch.empty(n_recv, dtype=torch.int32, device=item.device)
            self._a2a(self.recv_ids, st["send_ids"][:n_send], rc, sc)
        reply = torch.empty((n_recv, self.d), dtype=self.row_dtype, device=item.device)
        if before_gather is not None and sparse.get("map") is not None:
            self.k.owner_claim(self.recv_ids, sparse["map"], sparse["slot_row"], self.rank)
            before_gather(n_recv)
            self.k.owner_gather(self.recv_ids, E_local, reply, None, None, self.rank, self.d)
        else:
            self.k.owner_gather(self.recv_ids, E_local, reply, sparse["map"], sparse["slot_row"], self.rank, self.d)
        self.rows_buf = self._grow(self.rows_buf, n_send)
        rows = self.rows_buf[:n_send]
        self._a2a(rows, reply, sc, rc)
        return rows

    def _grow(self, buf, n):
        if buf is None or buf.shape[0] < n:
            cap = max(n, self.B * (self.L + 1))
            buf = _lib.persistent(lambda: torch.empty((cap, self.d), dtype=self.row_dtype, device=self.device))
        return buf

    def make_sendbuf(self) -> torch.Tensor:
        if self.fc_active:
            self.send_buf = self.fc_send
            return self.fc_send
        self.send_buf = self._grow(self.send_buf, sum(self.send_counts))
        return self.send_buf[:sum(self.send_counts)]

    def backward(self, sendbuf: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Returns the owner's received gradient rows [n_recv, d] f32 (entry i <-> recv_ids[i]),
        written into `out` (>= n_recv rows, e.g. a deferred-gradient ring slot) when given."""
        self.backward_start(sendbuf, out)
        return self.backward_finish()

    def backward_start(self, sendbuf: torch.Tensor, out: Optional[torch.Tensor] = None, early: bool = False) -> None:
        """Issue the gradient-row all-to-all now, asynchronously on the process group's own stream
        (the caller's stream goes on with other work); backward_finish() makes the caller's stream
        wait for it and widens bf16 wire rows."""
        n_recv = self.n_recv
        if self.fc_active and out is None:
            # fixed-capacity form: the rows land in the fixed wire buffer (the caller moves them into
            # a device-chosen ring slot, fbn_ring_slot, or widens them itself)
            grad = wire = self.fc_wire
        else:
            grad = out[:n_recv] if out is not None else \
                torch.empty((n_recv, self.d), dtype=torch.float32, device=sendbuf.device)
            # (rows of the send buffer's dtype land in `out` directly: f32, or a bf16 ring slot)
            wire = grad if sendbuf.dtype == grad.dtype else \
                (self.fc_wire if self.fc_active else
                 torch.empty((n_recv, self.d), dtype=sendbuf.dtype, device=sendbuf.device))
        work = None
        if self.comm is not None and early:
            # RCCL on a stream of its own, right after the fields backward: the exchange runs beside
            # the rest of the backward (the grouped weight gradients); backward_finish() joins it
            cur = torch.cuda.current_stream(sendbuf.device)
            if self._comm_stream is None:
                self._comm_stream = torch.cuda.Stream(device=sendbuf.device)
            cs = self._comm_stream
            _lib.wait_stream(cs, cur)
            with torch.cuda.stream(cs):
                if self.fc_active:
                    self._a2a_fc(wire, sendbuf)
                else:
                    self._a2a(wire, sendbuf, self.recv_counts, self.send_counts)
            work = torch.cuda.Event()
            _lib.record_event(work, cs)
            for t in (wire, grad, sendbuf):
                t.record_stream(cs)
        elif self.fc_active:
            self._a2a_fc(wire, sendbuf)
        elif self.stage_on_cpu or self.comm is not None:       # host-staged, or on this stream
            self._a2a(wire, sendbuf, self.recv_counts, self.send_counts)
        else:
            work = dist.all_to_all_single(wire, sendbuf, self.recv_counts, self.send_counts, group=self.group,
                                          async_op=True)
        self._pending = (work, wire, grad)

    def backward_finish(self) -> torch.Tensor:
        work, wire, grad = self._pending
        self._pending = None
        if isinstance(work, torch.cuda.Event):              # native RCCL on the exchange's own stream
            _lib.wait_event(torch.cuda.current_stream(grad.device), work)
        elif work is not None:
            work.wait()
        if wire is not grad:
            self.k.widen(wire, grad)
        return grad


class DistCollective:
    """SyncBN / gradient all-reduce hook for ops.forward/backward (sum over ranks).

    det (deterministic mode): the sum is an all-gather followed by the ranks' slices added in rank
    order (fbn_sum_slices; a Python loop for CPU tensors) -- the same bits on every rank, from run to
    run and on either collective path (native RCCL or torch.distributed), where ncclAllReduce's order
    follows the reduction algorithm RCCL picks for the communicator."""

    def __init__(self, world: int, group=None, stage_on_cpu: bool = False, comm: Optional[NativeComm] = None,
                 det: bool = False):
        self.world = world
        self.group = group
        self.stage_on_cpu = stage_on_cpu
        self.comm = comm
        self.det = det
        self._gbuf = {}

    def _allreduce_det(self, t: torch.Tensor) -> None:
        n, w = t.numel(), self.world
        flat = t.view(-1)
        if not t.is_cuda:
            parts = [torch.empty_like(flat) for _ in range(w)]
            dist.all_gather(parts, flat, group=self.group)
            acc = parts[0].clone()
            for q in parts[1:]:
                acc += q
            flat.copy_(acc)
            return
        key = (n, t.dtype, t.device)
        buf = self._gbuf.get(key)
        if buf is None:
            buf = self._gbuf[key] = _lib.persistent(lambda: torch.empty(w * n, dtype=t.dtype, device=t.device))
        if self.comm is not None:
            self.comm.allgather(buf, flat)
        elif self.stage_on_cpu:
            parts = [torch.empty(n, dtype=t.dtype) for _ in range(w)]
            dist.all_gather(parts, flat.cpu(), group=self.group)
            buf.copy_(torch.cat(parts))
        else:
            dist.all_gather_into_tensor(buf, flat, group=self.group)
        call("fbn_sum_slices", ptr(buf), w, n, {torch.float32: 0, torch.float64: 1}[t.dtype], ptr(flat),
             _lib.stream_handle(t.device))

    def allreduce_(self, t: torch.Tensor) -> None:
        if self.world <= 1:
            return
        if self.det:
            self._allreduce_det(t)
            return
        if self.comm is not None:
            self.comm.allreduce_(t)
        elif self.stage_on_cpu:
            c = t.cpu()
            dist.all_reduce(c, group=self.group)
            t.copy_(c)
        else:
            dist.all_reduce(t, group=self.group)
