"""ctypes binding of libfibinet_hip.so (the C-ABI declared in include/fibinet.h).

The library is loaded once; a missing or un-loadable library raises immediately -- there is
no CPU fallback anywhere in the product path.  Every call goes through :func:`call`, which
raises ``RuntimeError`` with ``fbn_last_error()`` on a non-zero return code.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import struct
import threading
from typing import Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FBN_LIB_PATH") or os.path.join(_HERE, "libfibinet_hip.so")   # override: tuning tools

P = ctypes.c_void_p
I = ctypes.c_int
LL = ctypes.c_longlong
F = ctypes.c_float
D = ctypes.c_double
SZ = ctypes.c_size_t
U = ctypes.c_uint

# name -> (restype, argtypes); the single source of truth mirrored by include/fibinet.h
SIGNATURES = {
    "fbn_version": (I, []),
    "fbn_last_error": (ctypes.c_char_p, []),
    "fbn_device_ok": (I, []),
    "fbn_gemm_workspace_size": (SZ, [I, I, I, I]),
    "fbn_gemm": (I, [P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, I, F, I, I, I, P, P, SZ, P]),
    "fbn_gemm_split": (I, [P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, F, P, P, SZ, P, I, I, P, I, I, P]),
    "fbn_gemm_bf16out": (I, [P, P, P, I, I, I, I, I, I, I, I, P]),
    "fbn_gemm_s3": (I, [P, P, P, I, I, I, I, I, I, I, I, LL, LL, F, P, SZ, P]),
    "fbn_gemm_bn_bwd_part_supported": (I, [I, I, I, I, I, I, I]),
    "fbn_gemm_bn_bwd_part": (I, [P, P, P, I, I, I, I, I, I, I, I, P, P, P, F, P, P]),
    "fbn_bn_tile_stats": (I, [P, I, I, P, P, P]),
    "fbn_bn_tile_moments": (I, [P, I, I, P, P]),
    "fbn_bn_moments_finalize": (I, [P, D, I, P, P, P, P, F, F, I, P]),
    "fbn_bn_tile_finalize": (I, [P, I, I, D, P, P, P, P, F, F, I, P]),
    "fbn_bn_colpart_size": (SZ, [I, I]),
    "fbn_row_chunks": (I, [I]),
    "fbn_bn_bwd_chunks": (I, [I, I]),
    "fbn_bn_bwd_fused": (I, [P, P, P, P, P, F, P, P, P, P, I, I, D, P, P, P, P, P, P, P, P, P]),
    "fbn_bn_bwd_fused_img": (I, [P, P, P, P, P, F, P, P, P, P, I, I, D, P, P, P, P, P, P, P, P, P]),
    "fbn_colsum_partial": (I, [P, I, I, I, P, P]),
    "fbn_sum_jobs": (I, [P, I, P]),
    "fbn_sum_jobs2": (I, [P, I, P, I, P]),
    "fbn_gemm_slabs_size": (SZ, [I, I, I]),
    "fbn_gemm_slabs": (I, [P, P, I, I, I, I, I, I, I, P, SZ, P, I, I, P, I, I, P, P]),
    "fbn_gemm_slabs_split": (I, [I, I, I]),
    "fbn_gemm_slabs_group": (I, [P, I, P]),
    "fbn_gemm_slabs_group_split": (I, [I, I, I]),
    "fbn_fields_fwd": (I, [P, P, P, P, P, P, P, F, P, I, P, LL, P, P, P, P, P, I, P, P, P, P, I, I, P, P, P, P, P, I, I, I, I,
                           P]),
    "fbn_fields_fwd_hot": (I, [P, P, P, P, P, P, P, F, P, I, P, LL, P, P, P, P, I, P, P, P, P, I, I, P, P, P, P, P,
                               I, I, I, P, P, I, P]),
    "fbn_hot_rows": (I, [P, P, I, I, LL, P, P, P, I, I, I, P]),
    "fbn_fields_bwd_partials_size": (I, [I, I, I]),
    "fbn_fields_bwd_grid": (I, [I, I]),
    "fbn_fields_bwd": (I, [P, P, P, P, P, P, P, F, P, P, P, I, I, P, P, P, P, P, P, P, P, P, P, P, P, LL, P, P, I, I,
                           I, I, P]),
    "fbn_fields_bwd_img": (I, [P, P, P, P, P, P, P, F, P, P, P, I, I, P, P, P, P, P, P, P, P, P, P, P, P, LL, P, P, I,
                               I, I, I, P]),
    "fbn_pairs_fwd": (I, [P, P, P, P, I, I, I, I, I, P]),
    "fbn_pairs_bwd": (I, [P, P, P, P, P, P, P, I, I, I, I, P]),
    "fbn_pairs_fwd_img": (I, [P, P, P, P, I, I, I, P]),
    "fbn_pairs_bwd_img": (I, [P, P, P, P, P, I, I, I, P]),
    "fbn_bn_workspace_size": (SZ, [I, I]),
    "fbn_bn_stats_pass": (I, [P, I, I, P, P, P, P]),
    "fbn_bn_mean": (I, [P, D, I, P, P]),
    "fbn_bn_finalize": (I, [P, P, D, I, P, P, P, P, F, F, I, P]),
    "fbn_bn_stats": (I, [P, I, I, P, P, P, P, F, F, I, P, P]),
    "fbn_bn_eval_params": (I, [P, P, P, P, I, F, P]),
    "fbn_bn_act_fwd": (I, [P, P, I, I, P, P, P, P, F, P, U, P, P, P, P]),
    "fbn_bn_act_fwd_img": (I, [P, P, I, I, P, P, P, P, F, P, U, P, P, P, P]),
    "fbn_bn_act_head_fwd": (I, [P, P, I, I, P, P, P, P, F, P, U, P, P, P, P, P, P, P, P, P, F, P, F, P]),
    "fbn_bn_bwd_reduce": (I, [P, P, P, P, F, P, P, I, I, P, P, P]),
    "fbn_bn_bwd_apply": (I, [P, P, P, P, F, P, P, P, P, I, I, P, D, P, P, P, P, P, P, P]),
    "fbn_convert_bf16": (I, [P, I, P]),
    "fbn_bn_bwd": (I, [P, P, P, P, F, P, P, P, P, I, I, P, P, P, P, P, P]),
    "fbn_colsum_workspace_size": (SZ, [I, I]),
    "fbn_colsum": (I, [P, I, I, I, P, F, P, P]),
    "fbn_head_fwd": (I, [P, P, P, I, I, P, P, P, P, P, F, P]),
    "fbn_sigmoid_bwd": (I, [P, P, P, I, P]),
    "fbn_outer": (I, [P, P, P, I, I, P]),
    "fbn_sum": (I, [P, I, P, F, P]),
    "fbn_sumsq": (I, [P, LL, P, I, P, P]),
    "fbn_clip_coef": (I, [P, F, P, P, P]),
    "fbn_adam_dense": (I, [P, P, P, P, LL, P, P, P, F, F, F, P, F, P, P, P]),
    "fbn_sparse_fixup": (I, [P, P, P, I, I, LL, I, P, P, P, P, I, I, P]),
    "fbn_sumsq_sparse": (I, [P, P, P, I, I, I, P, P]),
    "fbn_sparse_fixup_dup": (I, [P, I, P, P, P, I, I, P]),
    "fbn_sumsq_sparse_norms": (I, [P, P, P, P, I, I, I, P, P, P, LL, P]),
    "fbn_sparse_fold_fx": (I, [P, P, I, P, P, I, I, P, P]),
    "fbn_adam_table": (I, [P, P, P, LL, I, P, P, P, P, I, P, P, P, F, F, F, I, P]),
    "fbn_adam_touched": (I, [P, P, P, I, P, P, P, P, I, I, P, P, P, F, F, F, P, P]),
    "fbn_adam_catchup": (I, [P, P, P, LL, I, P, I, P, I, I, P, P, P, F, F, F, P, P, P, LL, I, I, P]),
    "fbn_adam_claim_catchup": (I, [P, P, I, I, LL, P, P, P, P, P, P, P, P, LL, I, I, P, P, P, F, F, F, P, P, P, LL, I,
                                   I, P]),
    "fbn_adam_claim_catchup_conv": (I, [P, P, I, I, LL, P, P, P, P, P, P, P, P, LL, I, I, P, P, P, F, F, F, P, P, P,
                                        LL, I, I, P, I, P]),
    "fbn_adam_flush": (I, [P, P, P, LL, I, P, P, P, F, F, F, P, P, P, LL, I, I, P]),
    "fbn_adam_prefetch_rows": (I, [P, I, I, LL, P, P, P, P, P, I, P, P, P, F, F, F, P, P, P, LL, I, I, P]),
    "fbn_adam_prefetch": (I, [P, P, I, I, LL, P, P, P, P, P, I, P, P, P, F, F, F, P, P, P, LL, I, I, P]),
    "fbn_adam_prefetch_binned_ws_size": (SZ, [LL]),
    "fbn_adam_prefetch_binned": (I, [P, P, I, I, LL, P, P, P, P, P, I, P, P, P, F, F, F, P, P, P, LL, I, I, P, SZ, P]),
    "fbn_adam_selftest": (I, [I, ctypes.c_uint, P, P]),
    "fbn_adam_step_tail": (I, [P, P, P, P, LL, P, F, P, P, P, P, P, I, P, P, P, P, I, I, P, P, F, F, F, P, P, P, P, I,
                               LL, I, P, P, P, P, I, P, P]),
    "fbn_adam_commit": (I, [P, P, P, I, P, P, P, P, I, I, P, P, P, F, F, F, P, P, P, P, I, I, P]),
    "fbn_claim_rows": (I, [P, P, I, I, LL, P, P, P, P, P]),
    "fbn_pack_extras": (I, [P, P, P, P]),
    "fbn_unpack_extras": (I, [P, P, P, P]),
    "fbn_unpack_sumsq": (I, [P, P, P, LL, P, P]),
    "fbn_step_end": (I, [P, P, P, P, P, I, P, P]),
    "fbn_route": (I, [P, P, I, I, LL, LL, I, P, P, P, P, P, P, P]),
    "fbn_route_fc": (I, [P, P, I, I, LL, LL, I, I, P, P, P, P, P]),
    "fbn_route_fc_status": (I, [P, P, I, I, I, P, P, P]),
    "fbn_ring_slot": (I, [P, I, LL, P, P, P, I, LL, P, LL, LL, P]),
    "fbn_owner_gather_self": (I, [P, I, P, P, P, P, I, I, I, P, I, I, P]),
    "fbn_adam_owner_claim_catchup": (I, [P, I, I, P, P, P, P, P, P, LL, I, I, P, P, P, F, F, F, P, P, P, LL, I, I,
                                         P]),
    "fbn_owner_fold": (I, [P, I, I, P, P, P, I, P, LL, LL, P, I, LL, P, P, P, I, P, P, P]),
    "fbn_sumsq_flagged": (I, [P, I, P, P, I, P, P, P, I, P]),
    "fbn_owner_claim": (I, [P, I, P, P, I, P]),
    "fbn_owner_gather": (I, [P, I, P, P, P, P, I, I, I, P]),
    "fbn_widen_bf16": (I, [P, P, LL, P]),
    "fbn_pad_routes": (I, [P, P, P, I, I, P, P]),
    "fbn_compact_routes": (I, [P, I, I, P, P, P]),
    "fbn_copy_jobs": (I, [P, P, P, I, P]),
    "fbn_bilinear_supported": (I, [I]),
    "fbn_bilinear_fwd": (I, [P, P, P, I, I, I, P]),
    "fbn_bilinear_bwd": (I, [P, I, I, P, P, P, P, P, I, I, P]),
    "fbn_collate": (I, [P, I, P, P, I, I, P, P, P, P, P, LL, P, P, I, P, P, P, P, P, P, P, P, P]),
    "fbn_collate_zero_if": (I, [P, LL, P, P]),
    "fbn_plan_create": (I, [P]),
    "fbn_plan_destroy": (I, [P]),
    "fbn_plan_size": (I, [P]),
    "fbn_plan_add_call": (I, [P, ctypes.c_char_p, P, I, P, I]),
    "fbn_plan_add_record": (I, [P, I, P]),
    "fbn_plan_add_wait": (I, [P, P, I]),
    "fbn_plan_run": (I, [P, P]),
    "fbn_plan_event_sync": (I, [P, I]),
    "fbn_probe_arm": (I, [I]),
    "fbn_probe_disarm": (I, []),
    "fbn_probe_elapsed": (F, [I]),
    "fbn_comm_load": (I, [ctypes.c_char_p]),
    "fbn_comm_id_bytes": (I, []),
    "fbn_comm_unique_id": (I, [P]),
    "fbn_comm_init": (I, [P, P, I, I]),
    "fbn_comm_destroy": (I, [P]),
    "fbn_comm_alltoallv": (I, [P, P, P, P, P, LL, P]),
    "fbn_comm_alltoall_peers": (I, [P, P, P, LL, P]),
    "fbn_comm_alltoall": (I, [P, P, P, LL, P]),
    "fbn_comm_allreduce": (I, [P, P, LL, I, P]),
    "fbn_comm_allgather": (I, [P, P, P, LL, P]),
    "fbn_sum_slices": (I, [P, I, LL, I, P, P]),
    "fbn_comm_watch": (I, [LL]),
    "fbn_comm_heartbeat": (I, [P]),
    "fbn_comm_abort": (I, [P]),
    "fbn_comm_watchdog_fired": (I, [P]),
}

_lib: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `python -m ctr_recommendation_amd.build` "
                "(the FiBiNET path has no CPU fallback)")
        h = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _lib = h
    return _lib


_fns = {}
_UNCHECKED = ("fbn_version", "fbn_device_ok", "fbn_probe_elapsed", "fbn_comm_watchdog_fired")
_tls = threading.local()           # .prog: the StepProgram recording on this thread (or None)


# FBN_DEBUG_SYNC=<path> (diagnostics only): every call is logged to <path> and followed by a device
# synchronize, so an asynchronous kernel fault surfaces at -- and is attributed to -- its own call
_DEBUG_SYNC = os.environ.get("FBN_DEBUG_SYNC")
_debug_log = None


def _debug_sync(name: str) -> None:
    global _debug_log
    if _debug_log is None:
        _debug_log = open(_DEBUG_SYNC, "a", buffering=1)
    _debug_log.write(name + "\n")
    torch.cuda.synchronize()


def call(name: str, *args) -> int:
    f = _fns.get(name)
    if f is None:                  # bound ctypes function, looked up once (host time per step)
        f = _fns[name] = getattr(lib(), name)
    if _DEBUG_SYNC:
        _debug_sync("> " + name)
    rc = f(*args)
    if _DEBUG_SYNC:
        _debug_sync("< " + name)
    if rc and isinstance(rc, int) and name not in _UNCHECKED and not name.endswith(("_size", "_grid")):
        msg = lib().fbn_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed (code {rc}): {msg}")
    prog = getattr(_tls, "prog", None)
    if prog is not None:
        prog.add_call(name, f, args)
    return rc


def keep(obj) -> None:
    """A host object whose address was passed to a call as an integer (a job array): kept alive
    by the step program being recorded, whose replays pass the same address again."""
    prog = getattr(_tls, "prog", None)
    if prog is not None:
        prog.keep.append(obj)


def recording() -> bool:
    return getattr(_tls, "prog", None) is not None


def persistent(fn):
    """fn() -- allocations that outlive the step (cached scratch, activation buffers, routing sets,
    state grown on first use) -- made OUTSIDE a step program's recording pool.  The pool holds the
    step's temporaries, whose blocks programs share once freed (steps never overlap); a buffer that
    lives on and took such a block would be overwritten by every replay of the program that recorded
    the temporary there.  Pool routing is per thread (torch.cuda.use_mem_pool), so while recording
    fn runs on a helper thread, on the caller's current stream."""
    prog = getattr(_tls, "prog", None)
    if prog is None:
        return fn()
    stream = torch.cuda.current_stream(prog.device)
    box = {}

    def run():
        try:
            torch.cuda.set_device(prog.device)
            with torch.cuda.stream(stream):
                box["out"] = fn()
        except BaseException as e:          # re-raised on the caller's thread
            box["err"] = e

    t = threading.Thread(target=run, name="fbn-persistent-alloc")
    t.start()
    t.join()
    if "err" in box:
        raise box["err"]
    return box["out"]


def pool_segments(pool) -> list:
    """[(start, end)) device address ranges of the segments a torch.cuda.MemPool owns (from the caching
    allocator's snapshot): the step programs' recording pool, for check_outside_pool()."""
    pid = tuple(pool.id)
    out = []
    for seg in torch.cuda.memory_snapshot():
        if tuple(seg.get("segment_pool_id", ())) == pid:
            out.append((int(seg["address"]), int(seg["address"]) + int(seg["total_size"])))
    return sorted(out)


def tensors_of(obj, _seen=None, _path="", _depth=0):
    """(path, tensor) for every device tensor reachable from obj through attributes, dicts, lists and
    tuples (the objects of this package only: a trainer, its exchange, routing sets, caches)."""
    seen = set() if _seen is None else _seen
    if id(obj) in seen or _depth > 8:
        return
    seen.add(id(obj))
    if isinstance(obj, torch.Tensor):
        if obj.is_cuda and obj.numel():
            yield _path, obj
        return
    if isinstance(obj, dict):
        for k, v in obj.items():
            yield from tensors_of(v, seen, f"{_path}[{k!r}]", _depth + 1)
    elif isinstance(obj, (list, tuple)):
        for i, v in enumerate(obj):
            yield from tensors_of(v, seen, f"{_path}[{i}]", _depth + 1)
    elif type(obj).__module__.startswith("ctr_recommendation_amd") and hasattr(obj, "__dict__"):
        for k, v in vars(obj).items():
            yield from tensors_of(v, seen, f"{_path}.{k}", _depth + 1)


def check_outside_pool(obj, pool) -> None:
    """The step programs' address-lifetime invariant: no tensor that outlives a step --
    anything reachable from obj (a trainer: its persistent state, its exchange's routing sets, its
    caches) -- may lie in the recording pool.  The pool hands its freed blocks to the next recording,
    and every replay of the program that recorded a temporary at such an address overwrites it (round
    5: the sharded fold buffer).  Raises RuntimeError naming the offending tensors."""
    segs = pool_segments(pool)
    bad = []
    for path, t in tensors_of(obj):
        lo = t.data_ptr()
        hi = lo + t.untyped_storage().nbytes()
        for a, b in segs:
            if lo < b and a < hi:
                bad.append(f"{path} [{lo:#x}, {hi:#x})")
                break
    if bad:
        raise RuntimeError("tensors that outlive the step lie in the step programs' recording pool "
                           "(allocate them through _lib.persistent): " + "; ".join(bad[:12]))


def wait_stream(dst, src) -> None:
    """dst.wait_stream(src), recorded as a stream edge while a step program is being recorded."""
    dst.wait_stream(src)
    prog = getattr(_tls, "prog", None)
    if prog is not None and dst.cuda_stream != src.cuda_stream:
        prog.edge(src.cuda_stream, dst.cuda_stream)


def record_event(ev, stream) -> None:
    """ev.record(stream) (recorded: the program's event slot of ev)."""
    ev.record(stream)
    prog = getattr(_tls, "prog", None)
    if prog is not None:
        call_raw("fbn_plan_add_record", prog.h, prog.slot_of(ev), stream.cuda_stream)


def wait_event(stream, ev) -> None:
    """stream.wait_event(ev) (recorded: a wait on the program's event slot of ev)."""
    stream.wait_event(ev)
    prog = getattr(_tls, "prog", None)
    if prog is not None:
        call_raw("fbn_plan_add_wait", prog.h, stream.cuda_stream, prog.slot_of(ev))


def call_raw(name: str, *args) -> int:
    """A call that is never recorded (the step-program API itself)."""
    f = _fns.get(name)
    if f is None:
        f = _fns[name] = getattr(lib(), name)
    rc = f(*args)
    if rc:
        msg = lib().fbn_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed (code {rc}): {msg}")
    return rc


_INT_TYPES = (P, I, LL, SZ, U)
_MASK64 = (1 << 64) - 1


def _as_u64(v) -> int:
    if v is None:
        return 0
    if isinstance(v, bool):
        return int(v)
    if isinstance(v, int):
        return v & _MASK64
    if isinstance(v, ctypes.c_void_p):
        return (v.value or 0) & _MASK64
    if isinstance(v, (ctypes.Array, ctypes.Structure)):
        return ctypes.addressof(v)
    if isinstance(v, ctypes._SimpleCData):
        return int(v.value) & _MASK64
    raise TypeError(f"step program: cannot record an argument of type {type(v).__name__} (pass an address)")


def _f32_in_f64(x: float) -> float:
    """The double whose low 32 bits are the float32 bits of x (a float argument in an xmm register)."""
    bits = struct.unpack("<I", struct.pack("<f", x))[0]
    return struct.unpack("<d", struct.pack("<Q", bits))[0]


class KernelProbe:
    """The kernels of one entry-point call, timed on the device (bench.py's rooflines): opened right
    before the call (fbn_probe_arm), closed right after (fbn_probe_disarm); elapsed_time() is the
    span from the first kernel's start to the last one's end, as rocprofv3 sees them (the library
    launches every kernel with hipExtLaunchKernelGGL and the probe's event pair), or -1 when the call
    launched nothing.  While a step program is being recorded the arm / disarm are recorded calls:
    every replay re-arms the slot, so after a replay the slot holds that replay's span.  Same
    interface as a torch.cuda.Event pair's start.elapsed_time(end)."""
    _next = 0

    def __init__(self):
        self.slot = KernelProbe._next
        KernelProbe._next += 1
        (call if recording() else call_raw)("fbn_probe_arm", self.slot)

    def done(self) -> None:
        (call if recording() else call_raw)("fbn_probe_disarm")

    def elapsed_time(self, _end=None) -> float:
        return float(lib().fbn_probe_elapsed(self.slot))


class StepProgram:
    """A recorded training step replayed by the native step driver (csrc/plan.cpp, include/fibinet.h
    "step programs").  Record with ``with prog.recording(): <run the step eagerly>``; every call()
    on this thread is appended (after it ran), wait_stream / record_event / wait_event become the
    program's stream edges, and every device allocation goes to the program's private memory pool,
    so the addresses the recorded calls name stay owned by the program (the pool is used by
    recordings only; steps never overlap, so programs may share its freed blocks, as torch's graphs
    share a pool).  run() replays the whole step with one host call."""

    def __init__(self, device=None):
        h = ctypes.c_void_p()
        call_raw("fbn_plan_create", ctypes.byref(h))
        self.h = h.value
        self.device = torch.device(device if device is not None else "cuda")
        self.keep = []
        self._slots = {}
        self._nslot = 0
        self.pool = None
        self._failed = ctypes.c_int(-1)
        self._run = lib().fbn_plan_run

    def add_call(self, name, f, args) -> None:
        types = SIGNATURES[name][1]
        ints, flts = [], []
        for t, v in zip(types, args):
            if t is F:
                flts.append(_f32_in_f64(float(v)))
            elif t is D:
                flts.append(float(v))
            else:
                ints.append(_as_u64(v))
                if isinstance(v, (ctypes.Array, ctypes.Structure, ctypes.c_void_p)):
                    self.keep.append(v)
        ia = (ctypes.c_ulonglong * max(1, len(ints)))(*ints)
        fa = (ctypes.c_double * max(1, len(flts)))(*flts)
        call_raw("fbn_plan_add_call", self.h, name.encode(), ia, len(ints), fa, len(flts))

    def slot_of(self, ev) -> int:
        k = id(ev)
        if k not in self._slots:
            self._slots[k] = self._nslot
            self._nslot += 1
            self.keep.append(ev)           # id() stays unique while the event lives
        return self._slots[k]

    def edge(self, src_stream: int, dst_stream: int) -> None:
        slot = self._nslot
        self._nslot += 1
        call_raw("fbn_plan_add_record", self.h, slot, src_stream)
        call_raw("fbn_plan_add_wait", self.h, dst_stream, slot)

    @contextlib.contextmanager
    def recording(self, pool=None):
        if getattr(_tls, "prog", None) is not None:
            raise RuntimeError("a step program is already being recorded on this thread")
        self.pool = pool if pool is not None else torch.cuda.MemPool()
        _tls.prog = self
        try:
            with torch.cuda.use_mem_pool(self.pool, device=self.device):
                yield self
        finally:
            _tls.prog = None

    def __len__(self) -> int:
        return call_raw("fbn_plan_size", self.h) if False else lib().fbn_plan_size(self.h)

    def run(self) -> None:
        rc = self._run(self.h, ctypes.byref(self._failed))
        if rc:
            msg = lib().fbn_last_error().decode(errors="replace")
            raise RuntimeError(f"step program op {self._failed.value} failed (code {rc}): {msg}")

    def __del__(self):
        h, self.h = getattr(self, "h", None), None
        if h and _lib is not None:
            _lib.fbn_plan_destroy(h)


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device: Optional[torch.device] = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_hip(t: torch.Tensor, what: str = "input") -> None:
    if t.device.type != "cuda":
        raise RuntimeError(
            f"{what} is on {t.device}; the MI355X FiBiNET path runs only on a HIP device "
            "(no CPU fallback: move the model and batch with .to('cuda'))")
