"""Kernel sequencing for one FiBiNET forward / backward on a HIP device.

This module owns no math: every arithmetic step is a call into libfibinet_hip.so.  Torch is
used for device allocation and the current stream only.  Both the drop-in ``MM_FiBiNET``
(autograd) and the native ``FiBiNETTrainer`` drive these two functions.

Layouts (B = batch, d = embedding dim, L = history length; DESIGN.md "HBM layout"):
  c      [B, 15d]  compact MLP input [V_1..V_5 | p_12..p_45]; the 6d structurally-zero
                   columns of the reference's 21d input (V_0 and pairs (0,j)) are never stored:
                   weight column k' of the compact layout is column remap(k') of mlp.0.weight,
                   remap = k' + (k' < 5d ? d : 6d).
  Vc, X  [B, 5, d] fields 1..5 after / before SENET;  U [B, 5, d] = Vc W.
  hmm    [B, d]    mm projection before LayerNorm.
"""
from __future__ import annotations

import os

import ctypes
from dataclasses import dataclass
from typing import Dict, Optional

import torch

from . import _lib
from ._lib import call, ptr

INT_MAX = 0x7FFFFFFF
NO_REMAP = (INT_MAX, 0, 0)
H1, H2 = 512, 256
LN_EPS = 1e-5
BN_EPS = 1e-5
BN_MOMENTUM = 0.1


# the trainer's BN2 backward first pass inside the forward head kernel (A/B knob)
_BN2_BWD_IN_FWD = os.environ.get("FBN_BN2_BWD_IN_FWD", "1") == "1"
# bf16_fwd: the backward's fp32 GEMMs as split-bf16 x3 (fbn_gemm bf16 = 2) with FBN_SPLIT_BWD=1 (A/B knob)
_SPLIT_BWD = os.environ.get("FBN_SPLIT_BWD", "0") == "1"
# bf16_fwd: the backward's GEMMs as ONE bf16 GEMM over 3 K each, on split operand images made once
# (fbn_convert_bf16 part 2 / 3: [hi, hi, lo] x [hi, lo, hi]) -- the LDS-DMA bf16 path instead of the
# fp32 MFMA (FBN_SPLIT3=0: fp32 MFMA, A/B)
_SPLIT3 = os.environ.get("FBN_SPLIT3", "1") != "0"
# bf16, one process: the BN1 backward first pass inside the epilogue of its dgrad GEMM (A/B knob)
_BN1_BWD_IN_GEMM = os.environ.get("FBN_BN1_BWD_IN_GEMM", "1") == "1"


def wa_remap(d: int):
    """compact MLP-input column -> mlp.0.weight column (skips V_0 and the five (0,j) pairs)."""
    return (5 * d, d, 6 * d)


def _ws(nbytes: int, device) -> Optional[torch.Tensor]:
    if nbytes <= 0:
        return None
    return torch.empty((nbytes + 7) // 8, dtype=torch.float64, device=device)


def gemm(A, B, C, M, N, K, lda, ldb, ldc, transA, transB, bias=None, rB=NO_REMAP, rC=NO_REMAP, beta=0.0,
         bf16=False, stream=None, stats=None):
    """C = op(A) op(B) (+bias, +beta C).  A / B may be fp32 or bf16 (torch.bfloat16) tensors."""
    nbytes = _lib.lib().fbn_gemm_workspace_size(M, N, K, int(bf16))
    ws = _ws(nbytes, C.device)
    a16, b16 = int(A.dtype == torch.bfloat16), int(B.dtype == torch.bfloat16)
    call("fbn_gemm", ptr(A), ptr(B), ptr(C), ptr(bias), M, N, K, lda, ldb, ldc, int(transA), int(transB),
         rB[0], rB[1], rB[2], rC[0], rC[1], rC[2], float(beta), int(bf16 or a16 or b16), a16, b16, ptr(stats),
         ptr(ws), nbytes,
         stream if stream is not None else _lib.stream_handle())


def _probe_start(probe, name):
    """bench probes: a kernel-span probe (_lib.KernelProbe) armed for the next library call."""
    if probe is None:
        return None
    kp = _lib.KernelProbe()
    probe.setdefault(name, []).append((kp, None))
    return kp


def _probe_end(kp) -> None:
    if kp is not None:
        kp.done()


def fused_bilinear(d: int) -> bool:
    """bf16 "all" bilinear as one fused MFMA + pair-product launch each way (csrc/bilinear.hip);
    FBN_NO_FUSED_BILINEAR=1 selects the GEMM + pair-kernel path (A/B measurements)."""
    return os.environ.get("FBN_NO_FUSED_BILINEAR") != "1" and bool(_lib.lib().fbn_bilinear_supported(d))


def split_mlp_input(d: int) -> bool:
    """bf16 MLP-input GEMMs read [Vc16 | pair block of c] as a split operand (LDS-DMA path:
    the 5d-column boundary must be a multiple of 128)."""
    return (5 * d) % 128 == 0


def wa_ld(d: int) -> int:
    """Row stride of the bf16 Wa image and of the bf16 MLP input c: 15d, or -- when 15d is not a
    multiple of 64 and c is not a split operand (d = 16: 240) -- 15d rounded up to 64 with zero
    columns, so the layer-1 GEMM takes the LDS-DMA path over K = 256 instead of the generic kernel
    over K = 240 (C2)."""
    kc = 15 * d
    return kc if (kc % 64 == 0 or split_mlp_input(d)) else (kc + 63) // 64 * 64


def gemm_split(A, B, C, M, N, K, lda, ldb, ldc, transA, transB, bias=None, rC=NO_REMAP, beta=0.0, stream=None,
               stats=None, A2=None, lda2=0, kseg=INT_MAX, B2=None, ldb2=0, nseg=INT_MAX):
    """bf16 C = op(A) op(B) with A = [A | A2] along K (k-contiguous A) or B = [B | B2] along N (k-major B)."""
    nbytes = _lib.lib().fbn_gemm_workspace_size(M, N, K, 1)
    ws = _ws(nbytes, C.device)
    call("fbn_gemm_split", ptr(A), ptr(B), ptr(C), ptr(bias), M, N, K, lda, ldb, ldc, int(transA), int(transB),
         rC[0], rC[1], rC[2], float(beta), ptr(stats), ptr(ws), nbytes, ptr(A2), lda2, kseg, ptr(B2), ldb2, nseg,
         stream if stream is not None else _lib.stream_handle())


class _ConvJob(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("rows", ctypes.c_int), ("cols", ctypes.c_int),
                ("ld", ctypes.c_int), ("trans", ctypes.c_int), ("seg", ctypes.c_int), ("off0", ctypes.c_int),
                ("off1", ctypes.c_int), ("part", ctypes.c_int), ("dld", ctypes.c_int), ("pst", ctypes.c_int)]
CONV_MAX = 16   # include/fibinet.h: jobs per fbn_convert_bf16 launch


def split_images(specs, stream) -> None:
    """ONE fbn_convert_bf16 launch (part 2) of split-bf16 operand images: specs = [(src, dst, rows,
    cols, ld, trans, remap)], dst [2, rows, cols] bf16 = (hi, lo) of the fp32 source (bf16_fwd
    backward: fbn_gemm_s3 and the split-bf16 x3 slab GEMMs read A_hi B_hi + A_hi B_lo + A_lo B_hi)."""
    jobs = (_ConvJob * CONV_MAX)()
    _lib.keep(jobs)
    for i, (src, dst, rows, cols, ld, trans, rm) in enumerate(specs):
        jobs[i] = _ConvJob(src.data_ptr(), dst.data_ptr(), rows, cols, ld, trans, rm[0], rm[1], rm[2], 2, 0,
                           rows * cols)
    call("fbn_convert_bf16", ctypes.cast(jobs, ctypes.c_void_p).value, len(specs), stream)


def s3_ok(M, N, K0, lda, ldb, transA, transB) -> bool:
    """fbn_gemm_s3's LDS-DMA conditions."""
    return K0 % 64 == 0 and lda % 8 == 0 and ldb % 8 == 0 and (not transA or M % 8 == 0) and (transB or N % 8 == 0)


def gemm_s3(A, B, C, M, N, K0, lda, ldb, ldc, transA, transB, beta=0.0, stream=None):
    """C (+)= split-bf16 x3 product of the (hi, lo) images A [2, ...] and B [2, ...] (fbn_gemm_s3)."""
    nbytes = _lib.lib().fbn_gemm_workspace_size(M, N, 3 * K0, 1)
    ws = _ws(nbytes, C.device)
    call("fbn_gemm_s3", ptr(A), ptr(B), ptr(C), M, N, K0, lda, ldb, ldc, int(transA), int(transB), A[0].numel(),
         B[0].numel(), float(beta), ptr(ws), nbytes, stream if stream is not None else _lib.stream_handle())


def bf16_weights(p: Dict[str, torch.Tensor], d: int, a: Dict[str, torch.Tensor], stream,
                 x: Optional[torch.Tensor] = None, images: bool = False) -> Dict[str, torch.Tensor]:
    """bf16 images of the GEMM weights, laid out so every bf16 GEMM operand is K-contiguous:
    Wa_nz [512,15d] (zero columns dropped) and its transpose, Wb and Wb^T, W and W^T, Wp;
    plus x (the batch's item_emb_d128, [B,128]) when given -- all in one launch.  images (bf16_fwd
    training): Wa^T, Wb^T, W and x also get their lo image (a["s3w_<name>"] = [2, ...]: hi, lo), the
    split-bf16 x3 backward's operands, from the same read."""
    jobs, n, out = bf16_weight_jobs(p, d, a, x, images)
    call("fbn_convert_bf16", ctypes.cast(jobs, ctypes.c_void_p).value, n, stream)
    return out


def bf16_weight_jobs(p: Dict[str, torch.Tensor], d: int, a: Dict[str, torch.Tensor],
                     x: Optional[torch.Tensor] = None, images: bool = False):
    """(job records, count, images) of bf16_weights, for a launch that carries the conversion
    (fbn_convert_bf16, or the step head fbn_adam_claim_catchup_conv); the records live in a["_conv_jobs"]."""
    dev = p["mlp.0.weight"].device
    KC = 15 * d
    spec = [("Wa", p["mlp.0.weight"], H1, KC, 21 * d, 0, wa_remap(d)),
            ("WaT", p["mlp.0.weight"], KC, H1, 21 * d, 1, wa_remap(d)),
            ("Wb", p["mlp.4.weight"], H2, H1, H1, 0, NO_REMAP),
            ("WbT", p["mlp.4.weight"], H1, H2, H1, 1, NO_REMAP),
            ("Wp", p["mm_proj.0.weight"], d, 128, 128, 0, NO_REMAP)]
    if "bilinear.W" in p:
        spec += [("W", p["bilinear.W"], d, d, d, 0, NO_REMAP), ("WT", p["bilinear.W"], d, d, d, 1, NO_REMAP)]
    if x is not None:
        spec.append(("x", x, x.shape[0], x.shape[1], x.shape[1], 0, NO_REMAP))
    jobs = (_ConvJob * CONV_MAX)()
    a["_conv_jobs"] = jobs
    _lib.keep(jobs)               # its address is passed as an integer (step programs keep it alive)
    out = {}
    for i, (name, src, rows, cols, ld, trans, rm) in enumerate(spec):
        img = images and name in ("WaT", "WbT", "W", "x")
        key = ("s3w_" if img else "w16_") + name
        dld = wa_ld(d) if name == "Wa" else cols          # Wa: zero columns up to the GEMM's K (wa_ld)
        shape = (2, rows, cols) if img else (rows, dld)
        t = a.get(key)
        if t is None or tuple(t.shape) != shape:
            t = _lib.persistent(lambda: torch.zeros(shape, dtype=torch.bfloat16, device=dev))
            a[key] = t
        out[name] = t[0] if img else (t[:, :cols] if dld != cols else t)
        if name == "Wa":
            out["Wa_full"] = t                          # [H1, wa_ld(d)]: the layer-1 GEMM's operand
        jobs[i] = _ConvJob(src.data_ptr(), t.data_ptr(), rows, cols, ld, trans, rm[0], rm[1], rm[2],
                           2 if img else 0, dld if dld != cols else 0, rows * cols if img else 0)
    return jobs, len(spec), out


class _SumJob(ctypes.Structure):
    _fields_ = [("part", ctypes.c_void_p), ("out", ctypes.c_void_p), ("nch", ctypes.c_int), ("C", ctypes.c_int),
                ("scale", ctypes.c_float), ("beta", ctypes.c_float), ("ld", ctypes.c_int), ("pad", ctypes.c_int)]


class _SlabJob(ctypes.Structure):
    _fields_ = [("ws", ctypes.c_void_p), ("out", ctypes.c_void_p), ("M", ctypes.c_int), ("N", ctypes.c_int),
                ("ldc", ctypes.c_int), ("nsplit", ctypes.c_int), ("seg", ctypes.c_int), ("off0", ctypes.c_int),
                ("off1", ctypes.c_int), ("beta", ctypes.c_float)]


# the weight-gradient GEMMs leave their split-K slabs for the step's one fbn_sum_jobs2 launch, and
# the fields backward its partial rows (FBN_DEFER_REDUCE=0: a reduce launch after each, A/B)
_DEFER_REDUCE = os.environ.get("FBN_DEFER_REDUCE", "1") != "0"
# ... and those GEMMs themselves wait for the end of the backward, where they run as ONE grouped
# launch (fbn_gemm_slabs_group) right before that sum launch (FBN_WGRAD_GROUP=0: each launched in
# place, A/B)
_WGRAD_GROUP = os.environ.get("FBN_WGRAD_GROUP", "1") != "0"


class _SlabGemm(ctypes.Structure):
    _fields_ = [("A", ctypes.c_void_p), ("B", ctypes.c_void_p), ("ws", ctypes.c_void_p), ("ws_bytes", ctypes.c_size_t),
                ("A2", ctypes.c_void_p), ("B2", ctypes.c_void_p), ("M", ctypes.c_int), ("N", ctypes.c_int),
                ("K", ctypes.c_int), ("lda", ctypes.c_int), ("ldb", ctypes.c_int), ("transA", ctypes.c_int),
                ("transB", ctypes.c_int), ("lda2", ctypes.c_int), ("kseg", ctypes.c_int), ("ldb2", ctypes.c_int),
                ("nseg", ctypes.c_int), ("s3k0", ctypes.c_int), ("lo_a", ctypes.c_longlong),
                ("lo_b", ctypes.c_longlong)]
_nsplit = ctypes.c_int(0)
# FBN_GATHER_HOT=<tau> (A/B variant of the gather, N1): rows a batch draws >= tau times staged in
# LDS per workgroup (fbn_hot_rows + fbn_fields_fwd_hot); 0 = off (default: measured slower)
_GATHER_HOT = int(os.environ.get("FBN_GATHER_HOT", "0"))


class DeferredSums:
    """Small reductions of one step, finalised together by ONE fbn_sum_jobs2 launch:
    out[c] = beta*out[c] + scale * sum_k part[k*ld + c], and the weight-gradient GEMMs' split-K
    slabs (gemm_slabs).  Partials must stay alive until flush()."""

    def __init__(self, cache: Optional[Dict[str, torch.Tensor]] = None):
        self.jobs = []
        self.slabs = []
        self.keep = []
        self.cache = cache      # slab workspaces kept across steps (one per GEMM shape)
        self.used = set()
        self.group = []         # slab GEMMs deferred to one fbn_gemm_slabs_group launch at flush()

    def add(self, part, nch, C, out, scale=1.0, beta=0.0, ld=0):
        self.jobs.append((part.data_ptr(), out.data_ptr(), int(nch), int(C), float(scale), float(beta), int(ld), 0))
        self.keep.append(part)

    def gemm_slabs(self, A, B, out, M, N, K, lda, ldb, ldc, transA, transB, rC=NO_REMAP, beta=0.0, stream=None,
                   A2=None, lda2=0, kseg=INT_MAX, B2=None, ldb2=0, nseg=INT_MAX, s3=False) -> bool:
        """out (+)= op(A) op(B) through fbn_gemm_slabs, its slabs summed at flush(); False (nothing
        launched) when the shape is outside the slab path's bf16 LDS-DMA conditions.  s3: A and B are
        (hi, lo) images [2, K, .] and the product is split-bf16 x3 over 3 K (grouped launch only)."""
        grouped = _WGRAD_GROUP and transA and not transB and A2 is None and M % 8 == 0 and N % 8 == 0
        if s3 and not (grouped and B2 is None and K % 64 == 0):
            return False
        lo_a, lo_b = (A[0].numel(), B[0].numel()) if s3 else (0, 0)
        K0, K = (K, 3 * K) if s3 else (0, K)
        if not (_DEFER_REDUCE and A.dtype == torch.bfloat16 and B.dtype == torch.bfloat16 and K % 64 == 0
                and lda % 8 == 0 and ldb % 8 == 0 and (not transA or M % 8 == 0) and (transB or N % 8 == 0)
                and N % 4 == 0 and ldc % 4 == 0 and all(x % 4 == 0 for x in rC[1:])
                and (rC[0] == INT_MAX or rC[0] % 4 == 0)):
            return False
        nbytes = _lib.lib().fbn_gemm_slabs_size(M, N, K)
        key = f"slab_ws_{M}_{N}_{K}"
        while key in self.used:       # two slab GEMMs of one shape in a step: separate workspaces
            key += "'"
        self.used.add(key)
        ws = self.cache.get(key) if self.cache is not None else None
        if ws is None or ws.numel() * 8 < nbytes:
            if self.cache is not None:
                ws = self.cache[key] = _lib.persistent(lambda: _ws(nbytes, out.device))
            else:
                ws = _ws(nbytes, out.device)
        st = stream if stream is not None else _lib.stream_handle()
        if grouped:
            # deferred to flush(): the step's weight gradients in one fbn_gemm_slabs_group launch
            # (their operands are not rewritten before it: stream order, buffers of this step)
            nsplit = _lib.lib().fbn_gemm_slabs_group_split(M, N, K)
            self.group.append((A.data_ptr(), B.data_ptr(), ws.data_ptr(), nbytes, 0, ptr(B2) or 0, M, N, K, lda,
                               ldb, 1, 0, 0, 0, ldb2, nseg if B2 is not None else INT_MAX, K0, lo_a, lo_b))
            self.keep += [A, B] + ([B2] if B2 is not None else [])
        else:
            call("fbn_gemm_slabs", ptr(A), ptr(B), M, N, K, lda, ldb, int(transA), int(transB), ptr(ws), nbytes,
                 ptr(A2), lda2, kseg, ptr(B2), ldb2, nseg, ctypes.addressof(_nsplit), st)
            nsplit = _nsplit.value
        self.slabs.append((ws.data_ptr(), out.data_ptr(), M, N, ldc, nsplit, rC[0], rC[1], rC[2], float(beta)))
        self.keep.append(ws)
        return True

    def colsum(self, X, B, C, ldx, out, stream):
        nch = _lib.lib().fbn_row_chunks(B)
        part = torch.empty((nch, C), dtype=torch.float32, device=X.device)
        call("fbn_colsum_partial", ptr(X), B, C, ldx, ptr(part), stream)
        self.add(part, nch, C, out)

    def launch_group(self, stream, probe: Optional[Dict[str, list]] = None, tstream=None) -> None:
        """The slab GEMMs recorded so far, in ONE fbn_gemm_slabs_group launch on `stream` (tstream: the
        torch stream of that handle, for the bench's events); their slabs are summed at flush()."""
        # (split-bf16 x3 problems and plain ones launch apart: a launch takes one kind)
        group = [x for x in self.group if x[-3]] + [x for x in self.group if not x[-3]]
        ev = _probe_start(probe, "wgrad_group") if group else None    # bench: the grouped launch
        while group:
            n = 0
            while n < min(6, len(group)) and bool(group[n][-3]) == bool(group[0][-3]):
                n += 1
            gc, group = group[:n], group[n:]
            garr = (_SlabGemm * len(gc))(*[_SlabGemm(*x) for x in gc])
            _lib.keep(garr)
            call("fbn_gemm_slabs_group", ctypes.addressof(garr), len(gc), stream)
        if ev is not None:
            _probe_end(ev)
            self.timed_group = True
        self.group = []

    timed_group = False

    def flush(self, stream, probe: Optional[Dict[str, list]] = None):
        # the bench's "wgrad_group" events time the launch of the step's weight gradients: the early one
        # when the trainer launched it beside the fields backward, else this one
        self.launch_group(stream, None if self.timed_group else probe)
        jobs, slabs = self.jobs, self.slabs
        while jobs or slabs:
            jc, sc = jobs[:16], slabs[:8]
            jobs, slabs = jobs[16:], slabs[8:]
            arr = (_SumJob * max(1, len(jc)))(*[_SumJob(*j) for j in jc])
            sarr = (_SlabJob * max(1, len(sc)))(*[_SlabJob(*j) for j in sc])
            _lib.keep((arr, sarr))
            call("fbn_sum_jobs2", ctypes.addressof(arr), len(jc), ctypes.addressof(sarr), len(sc), stream)
        self.jobs, self.slabs, self.keep = [], [], []
        self.used = set()


def colsum(X, B, C, ldx, out, beta=0.0, stream=None):
    ws = _ws(_lib.lib().fbn_colsum_workspace_size(B, C), X.device)
    call("fbn_colsum", ptr(X), B, C, ldx, ptr(out), float(beta), ptr(ws),
         stream if stream is not None else _lib.stream_handle())


@dataclass
class FwdConfig:
    d: int
    L: int
    training: bool
    p_drop: float
    bf16: bool = False
    # forward GEMM operands rounded to bf16 (fp32 accumulation), the rest of the forward and the
    # whole backward fp32 from fp32 activations (bf16 must be False)
    fwd16: bool = False
    bilinear_each: bool = False
    R: int = 3


class Collective:
    """Hook for SyncBN: sum a float64 device tensor over ranks in place (identity on 1 rank)."""

    world = 1

    def allreduce_(self, t: torch.Tensor) -> None:  # pragma: no cover - overridden for N > 1
        return None


NO_COLLECTIVE = Collective()


def bn_train_stats(h, B, C, mean, invstd, run_mean, run_var, ntot, coll: Collective, stream, tiles=None):
    """Training-mode BatchNorm statistics over the GLOBAL batch (SyncBN when coll.world > 1).
    tiles: per-64-row-tile (sum, M2) partials written by the producing GEMM (no pass over h)."""
    dev = h.device
    if tiles is not None and coll.world <= 1:
        call("fbn_bn_tile_finalize", ptr(tiles), B, C, float(ntot), ptr(mean), ptr(invstd), ptr(run_mean),
             ptr(run_var), BN_MOMENTUM, BN_EPS, 1 if run_mean is not None else 0, stream)
        return
    s = torch.empty(C, dtype=torch.float64, device=dev)
    mean_d = torch.empty(C, dtype=torch.float64, device=dev)
    if tiles is not None:
        # SyncBN: raw f64 moments, ONE all-reduce per layer
        mom = torch.empty(2 * C, dtype=torch.float64, device=dev)
        call("fbn_bn_tile_moments", ptr(tiles), B, C, ptr(mom), stream)
        coll.allreduce_(mom)
        call("fbn_bn_moments_finalize", ptr(mom), float(ntot), C, ptr(mean), ptr(invstd), ptr(run_mean),
             ptr(run_var), BN_MOMENTUM, BN_EPS, 1 if run_mean is not None else 0, stream)
        return
    else:
        ws = _ws(_lib.lib().fbn_bn_workspace_size(B, C), dev)
        call("fbn_bn_stats_pass", ptr(h), B, C, None, ptr(s), ptr(ws), stream)
        coll.allreduce_(s)
        call("fbn_bn_mean", ptr(s), float(ntot), C, ptr(mean_d), stream)
        call("fbn_bn_stats_pass", ptr(h), B, C, ptr(mean_d), ptr(s), ptr(ws), stream)
        coll.allreduce_(s)
    call("fbn_bn_finalize", ptr(s), ptr(mean_d), float(ntot), C, ptr(mean), ptr(invstd), ptr(run_mean),
         ptr(run_var), BN_MOMENTUM, BN_EPS, 1 if run_mean is not None else 0, stream)


def bn_backward(G, gvec, w, hact, scale, hpre, mean, invstd, gamma, B, C, ntot, dpre, dgamma, dbeta, dw,
                coll: Collective, stream, dpre16=None, bias_grad=None, sums: Optional[DeferredSums] = None,
                hact16=None, part_pre=None, tag: str = "", dpre_img=None):
    """BN (+ReLU/dropout) backward; bias_grad (with sums): the preceding Linear's bias gradient
    = column sums of dpre, finalised later by sums.flush().  tag names the layer ("bn1" / "bn2"):
    its cached workspace and bias-gradient partials are the layer's own, so two BatchNorm layers of
    one width never share the partial slab that sums.flush() reads at the end of the backward.

    Single process only: hact may be None with hact16 (the bf16 activation image; a matrix source
    G needs only its sign) and dpre may be None when dpre16 is given (bf16 mode: nothing reads the
    f32 gradient, the bias gradient comes from the apply's column partials).  dpre_img (single process,
    bf16_fwd): the bf16 output as split images [2, B, C] (hi, lo) instead of dpre16."""
    dev = hpre.device
    cache = sums.cache if sums is not None and sums.cache is not None else {}
    nws = _lib.lib().fbn_bn_workspace_size(B, C)
    key = tag or str(C)
    ws = cache.get(f"bn_ws_{key}") if nws > 0 else None
    if nws > 0 and (ws is None or ws.numel() * 8 < nws):
        ws = cache[f"bn_ws_{key}"] = _lib.persistent(lambda: _ws(nws, dev))
    if coll.world <= 1:
        part = None
        if bias_grad is not None:
            nch = _lib.lib().fbn_bn_bwd_chunks(B, C)
            part = cache.get(f"bn_part_{key}")
            if part is None or tuple(part.shape) != (nch, C):
                part = cache[f"bn_part_{key}"] = _lib.persistent(
                    lambda: torch.empty((nch, C), dtype=torch.float32, device=dev))
            sums.add(part, nch, C, bias_grad)
        call("fbn_bn_bwd_fused_img" if dpre_img is not None else "fbn_bn_bwd_fused", ptr(G), ptr(gvec), ptr(w),
             ptr(hact), ptr(hact16), float(scale), ptr(hpre), ptr(mean), ptr(invstd), ptr(gamma), B, C, float(ntot),
             ptr(dpre), ptr(dpre_img if dpre_img is not None else dpre16), ptr(dgamma), ptr(dbeta), ptr(dw), ptr(part),
             ptr(part_pre), ptr(ws), stream)
        return
    assert hact is not None and dpre is not None, "SyncBN backward reads the f32 activation and gradient"
    red = torch.empty(3 * C, dtype=torch.float64, device=dev)
    call("fbn_bn_bwd_reduce", ptr(G), ptr(gvec), ptr(w), ptr(hact), float(scale), ptr(hpre), ptr(mean), B, C,
         ptr(red), ptr(ws), stream)
    red_g = red
    if coll.world > 1:
        red_g = red.clone()
        coll.allreduce_(red_g)            # global sums -> the SyncBN input gradient
    call("fbn_bn_bwd_apply", ptr(G), ptr(gvec), ptr(w), ptr(hact), float(scale), ptr(hpre), ptr(mean), ptr(invstd),
         ptr(gamma), B, C, ptr(red_g), float(ntot), ptr(dpre), ptr(dpre16), ptr(dgamma), ptr(dbeta), ptr(dw), ptr(ws),
         stream)
    if coll.world > 1:
        # parameter grads from this rank's sums only (the dense-grad all-reduce adds the ranks);
        # B = 0 runs just the finalize step, after the apply above has consumed its coefficients
        call("fbn_bn_bwd_apply", ptr(G), ptr(gvec), ptr(w), ptr(hact), float(scale), ptr(hpre), ptr(mean),
             ptr(invstd), ptr(gamma), 0, C, ptr(red), float(ntot), None, None, ptr(dgamma), ptr(dbeta), ptr(dw),
             ptr(ws), stream)
    if bias_grad is not None:
        sums.colsum(dpre, B, C, C, bias_grad, stream)


def forward(p: Dict[str, torch.Tensor], batch: Dict[str, torch.Tensor], cfg: FwdConfig,
            rng: Optional[torch.Tensor] = None, *, table_rows: Optional[torch.Tensor] = None,
            pos: Optional[torch.Tensor] = None, sparse: Optional[Dict[str, torch.Tensor]] = None,
            err: Optional[torch.Tensor] = None, labels: Optional[torch.Tensor] = None,
            loss_denom: Optional[float] = None, coll: Collective = NO_COLLECTIVE, ntot: Optional[int] = None,
            masks_out: Optional[Dict[str, torch.Tensor]] = None, acts: Optional[Dict[str, torch.Tensor]] = None,
            probe: Optional[Dict[str, list]] = None, masks_in: Optional[Dict[str, torch.Tensor]] = None,
            after_gather=None, count_batches: bool = True, w16_ready: bool = False,
            hooks: Optional[Dict[str, object]] = None) -> Dict[str, torch.Tensor]:
    """Run the forward; returns the activation dict (probs, logits and what backward needs).

    p: parameter tensors keyed like the reference state_dict (fp32, contiguous, on device).
    table_rows/pos: multi-GPU mode (rows already exchanged); otherwise p['item_emb.weight'] is read.
    sparse: {'map','slot_row'} to register touched rows for the native sparse-grad Adam.
    labels: if given, fuses BCE: acts['loss_terms'] and acts['gout'] (= dL/dlogit).
    """
    d, L = cfg.d, cfg.L
    item_id = batch["item_id"]
    B = item_id.shape[0]
    dev = item_id.device
    st = _lib.stream_handle(dev)
    ntot = B if ntot is None else ntot
    f32 = dict(dtype=torch.float32, device=dev)
    a = acts if acts is not None else {}

    def buf(name, shape, dtype=torch.float32):
        t = a.get(name)
        if t is None or tuple(t.shape) != tuple(shape):
            t = _lib.persistent(lambda: torch.empty(shape, dtype=dtype, device=dev))
            a[name] = t
        return t

    seq = batch.get("item_seq", None)
    Lr = 0 if seq is None else L
    x_mm = batch["item_emb_d128"]
    bf = cfg.bf16
    f16 = cfg.fwd16 and not bf            # bf16 forward GEMM operands only
    g16 = bf or f16                       # the forward GEMMs take bf16 operands
    # w16_ready: the caller already converted this step's bf16 images (a["w16"]) on another stream
    # bf16_fwd training: the weight images carry their lo image too (the split-bf16 x3 backward)
    s3w = f16 and _SPLIT3 and cfg.training and not cfg.bilinear_each
    a["s3w"] = s3w and (not w16_ready or bool(a.get("w16_images")))   # (the trainer's images carry lo too)
    w16 = (a["w16"] if w16_ready else bf16_weights(p, d, a, st, x=x_mm, images=s3w)) if g16 else None
    a["w16"] = w16
    hmm = buf("hmm", (B, d))
    gemm(w16["x"] if g16 else x_mm, w16["Wp"] if g16 else p["mm_proj.0.weight"], hmm, B, d, 128, 128, 128, d, False,
         True, bias=p["mm_proj.0.bias"], bf16=g16, stream=st)
    if hooks and "after_mmproj" in hooks:         # trainer: side-stream work forked here
        hooks["after_mmproj"]()
    if hooks and "before_gather" in hooks:        # trainer: the table rows' claims ran on the side stream
        hooks["before_gather"]()
    X = buf("X", (B, 2, d))                     # fields 3 and 5 (the backward recomputes 1, 2, 4)
    # bf16 mode: the fields after SENET exist only as bf16 (GEMM operand and pair-kernel input)
    v16 = bf and not cfg.bilinear_each
    Vc = None if v16 else buf("Vc", (B, 5, d))
    Vc16 = buf("Vc16", (B, 5, d), torch.bfloat16) if v16 else None
    KC = 15 * d
    # bf16 mode: GEMM-only operand, rows wa_ld(d) apart (zero columns past 15d at d = 16)
    KCp = wa_ld(d) if bf else KC
    c = a.get("c")
    cdt = torch.bfloat16 if bf else torch.float32
    if c is None or tuple(c.shape) != (B, KCp) or c.dtype != cdt:
        c = a["c"] = _lib.persistent(lambda: torch.zeros((B, KCp), dtype=cdt, device=dev))
    # bf16 LDS-DMA mode: c's V block is never written -- the MLP GEMMs read [Vc16 | c[:, 5d:]] (split operand)
    split_c = v16 and split_mlp_input(d)
    a["split_c"] = split_c
    # bf16_fwd training whose split-bf16 x3 backward runs every GEMM on the LDS-DMA path: c and V exist
    # only as split images (fbn_pairs_fwd_img) -- no fp32 c is written or converted
    s3img = (f16 and _SPLIT3 and cfg.training and not cfg.bilinear_each and B % 64 == 0 and d % 64 == 0
             and _WGRAD_GROUP and _DEFER_REDUCE and coll.world <= 1)
    a["s3img"] = s3img
    if s3img:
        # V's split images: hi = the gather's bf16 copy (the U = V W GEMM's operand), lo from the
        # pair kernel
        a["s3_vc"] = buf("s3_vc_fwd", (2, 5 * B, d), torch.bfloat16)
        Vc16 = a["s3_vc"][0].view(B, 5, d)
    av = buf("a", (B, 6))
    cnt = buf("cnt", (B,))
    if err is None:
        err = buf("err", (1,), torch.int32)
        err.zero_()
    E = p["item_emb.weight"] if table_rows is None else table_rows
    V = p["item_emb.weight"].shape[0] if table_rows is None else 0
    sm = sparse or {}
    ev = _probe_start(probe, "fields_fwd")      # bench: the gather kernel's span
    if _GATHER_HOT and table_rows is None and V * d * 4 < 0xFFFFFF00:
        # A/B variant: the batch's rows drawn >= _GATHER_HOT times are staged in LDS per workgroup
        hc = a.get("hot_cnt")
        if hc is None or hc.numel() != V:
            hc = a["hot_cnt"] = _lib.persistent(lambda: torch.zeros(V, dtype=torch.int32, device=dev))
            a["hot_list"] = _lib.persistent(lambda: torch.zeros(256, dtype=torch.int32, device=dev))
            a["hot_n"] = _lib.persistent(lambda: torch.zeros(1, dtype=torch.int32, device=dev))
        H = 8192 // d
        call("fbn_hot_rows", ptr(item_id), ptr(seq) if Lr else None, B, Lr, V, ptr(hc), ptr(a["hot_list"]),
             ptr(a["hot_n"]), H, _GATHER_HOT, 0, st)
        call("fbn_fields_fwd_hot", ptr(item_id), ptr(seq) if Lr else None, ptr(batch["likes_level"]),
             ptr(batch["views_level"]), ptr(hmm), ptr(p["mm_proj.1.weight"]), ptr(p["mm_proj.1.bias"]), LN_EPS,
             ptr(p["cate_emb.weight"]), p["cate_emb.weight"].shape[0], ptr(E), V,
             ptr(p["senet.excitation.0.weight"]), ptr(p["senet.excitation.0.bias"]),
             ptr(p["senet.excitation.2.weight"]), ptr(p["senet.excitation.2.bias"]), cfg.R, ptr(X), ptr(Vc),
             ptr(Vc16), None if split_c else ptr(c), KCp, int(bf), ptr(av), ptr(cnt), ptr(err), ptr(sm.get("map")),
             ptr(sm.get("slot_row")), B, Lr, d, ptr(a["hot_list"]), ptr(a["hot_n"]), H, st)
        call("fbn_hot_rows", ptr(item_id), ptr(seq) if Lr else None, B, Lr, V, ptr(hc), None, ptr(a["hot_n"]), H,
             _GATHER_HOT, 1, st)
    else:
        call("fbn_fields_fwd", ptr(item_id), ptr(seq) if Lr else None, ptr(batch["likes_level"]),
             ptr(batch["views_level"]), ptr(hmm), ptr(p["mm_proj.1.weight"]), ptr(p["mm_proj.1.bias"]), LN_EPS,
             ptr(p["cate_emb.weight"]), p["cate_emb.weight"].shape[0], ptr(E), V, ptr(pos),
             ptr(p["senet.excitation.0.weight"]), ptr(p["senet.excitation.0.bias"]),
             ptr(p["senet.excitation.2.weight"]), ptr(p["senet.excitation.2.bias"]), cfg.R, ptr(X), ptr(Vc),
             ptr(Vc16), None if (split_c or s3img) else ptr(c), KCp,
             int(bf), ptr(av), ptr(cnt), ptr(err), ptr(sm.get("map")), ptr(sm.get("slot_row")), B, Lr, d,
             int(table_rows is not None and table_rows.dtype == torch.bfloat16), st)
    _probe_end(ev)
    if after_gather is not None:
        after_gather()
    if hooks and "after_fields" in hooks:         # trainer: side-stream work forked here
        hooks["after_fields"]()
    # bilinear: U = V W  ("all")  or  U_i = V_i W_i ("each"), then pair products into c
    fused_bil = bf and not cfg.bilinear_each and fused_bilinear(d)
    a["fused_bilinear"] = fused_bil
    if fused_bil:
        # one launch: MFMA U = V W in registers, pair products straight into c (U never stored)
        call("fbn_bilinear_fwd", ptr(Vc16), ptr(w16["WT"]), ptr(c), B, d, KCp, st)
    U = None if fused_bil else buf("U", (B, 5, d))
    if fused_bil:
        pass
    elif not cfg.bilinear_each:
        if bf:   # B(k,n) = W[k][n]: K-contiguous image is W^T
            gemm(Vc16, w16["WT"], U, 5 * B, d, d, d, d, d, False, True, bf16=True, stream=st)
        elif f16 and s3img:   # the gather's bf16 copy of the fields (= rounded on load), LDS-DMA path
            gemm(Vc16, w16["WT"], U, 5 * B, d, d, d, d, d, False, True, bf16=True, stream=st)
        elif f16:   # the fp32 fields rounded to bf16 on load
            gemm(Vc, w16["WT"], U, 5 * B, d, d, d, d, d, False, True, bf16=True, stream=st)
        else:
            gemm(Vc, p["bilinear.W"], U, 5 * B, d, d, d, d, d, False, False, stream=st)
    else:
        U.zero_()
        for f in range(1, 5):   # field index in Vc: f-1 <-> reference field f; W_list[f]
            gemm(Vc[:, f - 1], p[f"bilinear.W_list.{f}"], U[:, f - 1], B, d, d, 5 * d, d, 5 * d, False, False,
                 bf16=bf, stream=st)
    if s3img:
        a["s3_c"] = buf("s3_c_fwd", (2, B, KC), torch.bfloat16)
        call("fbn_pairs_fwd_img", ptr(Vc), ptr(U), ptr(a["s3_c"]), ptr(a["s3_vc"]), B, d, KC, st)
    elif not fused_bil:
        call("fbn_pairs_fwd", ptr(Vc), ptr(Vc16), ptr(U), ptr(c), B, d, KCp, int(cfg.bilinear_each), int(bf), st)
    # MLP layer 1
    h1pre = buf("h1pre", (B, H1))
    nt = (B + 63) // 64
    fuse = cfg.training
    t1 = buf("tiles1", (nt, H1, 2)) if fuse else None      # fused BN statistics (GEMM epilogue)
    t2 = buf("tiles2", (nt, H2, 2)) if fuse else None
    ev1 = _probe_start(probe, "gemm_mlp0")      # bench: the MLP's first GEMM
    if split_c:
        gemm_split(Vc16, w16["Wa"], h1pre, B, H1, KC, 5 * d, KC, H1, False, True, bias=p["mlp.0.bias"], stream=st,
                   stats=t1, A2=c[:, 5 * d:], lda2=KC, kseg=5 * d)
    elif f16 and _SPLIT3 and cfg.training and not cfg.bilinear_each:
        # bf16_fwd training: c's split images [hi; lo; hi] for the backward's GEMMs, made here -- the
        # GEMM takes the hi image (c rounded to bf16, as on load) through the LDS-DMA path
        if s3img:
            c2 = a["s3_c"]                          # fbn_pairs_fwd_img
        else:
            c2 = buf("s3_c_fwd", (2, B, KC), torch.bfloat16)
            split_images([(c, c2, B, KC, KC, 0, NO_REMAP)], st)
            a["s3_c"] = c2
        gemm(c2[0], w16["Wa_full"], h1pre, B, H1, KC, KC, wa_ld(d), H1, False, True, bias=p["mlp.0.bias"], bf16=True,
             stream=st, stats=t1)
    elif bf or f16:   # bf16_fwd: the fp32 MLP input rounded to bf16 on load
        a["s3_c"] = None
        # (bf16: K padded with zero columns to wa_ld(d) on both operands; bf16_fwd: fp32 c over K = 15d)
        gemm(c, w16["Wa_full"], h1pre, B, H1, KCp, KCp, wa_ld(d), H1, False, True, bias=p["mlp.0.bias"], bf16=True,
             stream=st, stats=t1)
    else:
        gemm(c, p["mlp.0.weight"], h1pre, B, H1, KC, KC, 21 * d, H1, False, True, bias=p["mlp.0.bias"],
             rB=wa_remap(d), stream=st, stats=t1)
    _probe_end(ev1)
    if hooks and "after_mlp0" in hooks:           # trainer: side-stream work forked here
        hooks["after_mlp0"]()
    mean1, inv1 = buf("mean1", (H1,)), buf("inv1", (H1,))
    mean2, inv2 = buf("mean2", (H2,)), buf("inv2", (H2,))
    h1 = buf("h1", (B, H1))
    h1_16 = buf("h1_16", (B, H1), torch.bfloat16) if g16 else None
    h2pre = buf("h2pre", (B, H2))
    h2 = buf("h2", (B, H2))
    p_drop = cfg.p_drop if cfg.training else 0.0
    m1 = masks_out.get("m1") if masks_out else None
    m2 = masks_out.get("m2") if masks_out else None
    mi1 = masks_in.get("m1") if masks_in else None
    mi2 = masks_in.get("m2") if masks_in else None
    if cfg.training:
        bn_train_stats(h1pre, B, H1, mean1, inv1, p["mlp.1.running_mean"], p["mlp.1.running_var"], ntot, coll, st,
                       tiles=t1)
    else:
        call("fbn_bn_eval_params", ptr(p["mlp.1.running_mean"]), ptr(p["mlp.1.running_var"]), ptr(mean1), ptr(inv1),
             H1, BN_EPS, st)
    # bf16, one process: the f32 activation has no reader (layer 2 and its weight gradient take
    # the bf16 image, the BN backward only its sign), so it is not written
    lean = (bf or s3img) and coll.world <= 1
    a["lean_h1"] = lean
    if s3img:
        # h1 only as split images: hi = the layer-2 GEMM operand, both = the split-bf16 x3 dWb operand;
        # the BN1 backward takes the ReLU / dropout mask from hi's sign
        a["s3_h1"] = buf("s3_h1_fwd", (2, B, H1), torch.bfloat16)
        h1_16 = a["s3_h1"][0]
        a["h1_16"] = h1_16
        call("fbn_bn_act_fwd_img", ptr(h1pre), None if lean else ptr(h1), B, H1, ptr(mean1), ptr(inv1),
             ptr(p["mlp.1.weight"]), ptr(p["mlp.1.bias"]), float(p_drop), ptr(rng), 1, ptr(m1), ptr(mi1),
             ptr(a["s3_h1"]), st)
    else:
        call("fbn_bn_act_fwd", ptr(h1pre), None if lean else ptr(h1), B, H1, ptr(mean1), ptr(inv1),
             ptr(p["mlp.1.weight"]), ptr(p["mlp.1.bias"]), float(p_drop), ptr(rng), 1, ptr(m1), ptr(mi1), ptr(h1_16),
             st)
    if g16:
        gemm(h1_16, w16["Wb"], h2pre, B, H2, H1, H1, H1, H2, False, True, bias=p["mlp.4.bias"], bf16=True, stream=st,
             stats=t2)
    else:
        gemm(h1, p["mlp.4.weight"], h2pre, B, H2, H1, H1, H1, H2, False, True, bias=p["mlp.4.bias"], stream=st,
             stats=t2)
    if cfg.training:
        bn_train_stats(h2pre, B, H2, mean2, inv2, p["mlp.5.running_mean"], p["mlp.5.running_var"], ntot, coll, st,
                       tiles=t2)
    else:
        call("fbn_bn_eval_params", ptr(p["mlp.5.running_mean"]), ptr(p["mlp.5.running_var"]), ptr(mean2), ptr(inv2),
             H2, BN_EPS, st)
    logits, probs = buf("logits", (B,)), buf("probs", (B,))
    lt = buf("loss_terms", (B,)) if labels is not None else None
    go = buf("gout", (B,)) if labels is not None else None
    # BN2 + ReLU + dropout with the head Linear(256,1) + sigmoid + BCE in the same launch; with the
    # labels (trainer, one BN group) also the first pass of the BN2 backward (its column partials)
    bpart = None
    if labels is not None and cfg.training and coll.world <= 1 and _BN2_BWD_IN_FWD:
        bpart = buf("bn2_bwd_part", (_lib.lib().fbn_bn_bwd_chunks(B, H2) * 3 * H2,), torch.float64)
    a["bn2_bwd_part"] = bpart
    bscale = 1.0 / (1.0 - cfg.p_drop) if (cfg.training and cfg.p_drop > 0) else 1.0   # = backward()'s scale
    call("fbn_bn_act_head_fwd", ptr(h2pre), ptr(h2), B, H2, ptr(mean2), ptr(inv2), ptr(p["mlp.5.weight"]),
         ptr(p["mlp.5.bias"]), float(p_drop), ptr(rng), 2, ptr(m2), ptr(mi2), ptr(p["mlp.8.weight"]),
         ptr(p["mlp.8.bias"]), ptr(logits), ptr(probs), ptr(labels), ptr(lt), ptr(go),
         float(loss_denom if loss_denom is not None else ntot), ptr(bpart), float(bscale), st)
    if cfg.training and count_batches and "mlp.1.num_batches_tracked" in p:
        p["mlp.1.num_batches_tracked"].add_(1)
        p["mlp.5.num_batches_tracked"].add_(1)
    a["err"] = err
    a["B"] = B
    return a


class _SideWork:
    """Weight-gradient GEMMs off the dgrad critical path: each is forked onto `side` once its
    operands exist (side waits for the main stream's work so far) and all are joined at the
    end of the backward.  Torch's current stream is `side` while they are issued, so their
    workspaces come from the side stream's allocator pool."""

    def __init__(self, side: Optional["torch.cuda.Stream"], dev):
        self.side = side
        self.dev = dev
        self.main = torch.cuda.current_stream(dev) if side is not None else None

    def run(self, fn):
        if self.side is None:
            fn(_lib.stream_handle(self.dev))
            return
        _lib.wait_stream(self.side, self.main)
        with torch.cuda.stream(self.side):
            fn(self.side.cuda_stream)

    def join(self):
        if self.side is not None:
            _lib.wait_stream(self.main, self.side)


def backward(p: Dict[str, torch.Tensor], batch: Dict[str, torch.Tensor], a: Dict[str, torch.Tensor],
             gout: torch.Tensor, g: Dict[str, torch.Tensor], cfg: FwdConfig, *,
             table_grad: Optional[torch.Tensor] = None, gvec: Optional[torch.Tensor] = None,
             gnorm: Optional[torch.Tensor] = None,
             pos: Optional[torch.Tensor] = None,
             sendbuf: Optional[torch.Tensor] = None, coll: Collective = NO_COLLECTIVE,
             ntot: Optional[int] = None, extra_sums=(), side: Optional["torch.cuda.Stream"] = None,
             probe: Optional[Dict[str, list]] = None, hooks: Optional[Dict[str, object]] = None) -> None:
    """Backward from dL/dlogit (gout [B]) into the gradient buffers ``g`` (same keys as ``p``).

    table_grad: dense [V, d] (drop-in, accumulated by atomics); or gvec [B, 2, d] (native
    trainer: per-sample {item-row grad, history-row grad}, resolved through the slot map)
    (native trainer); in multi-GPU mode (pos given) rows are written to sendbuf instead.
    Every g[...] buffer is overwritten (not accumulated), except the table gradient which is
    accumulated into (callers zero it).
    extra_sums: further (part, nch, C, out[, scale, beta]) reductions to finalise in the same
    fbn_sum_jobs launch as the bias gradients (the trainer's mean loss).
    side: optional stream for the weight-gradient GEMMs (overlap with the dgrad chain).  Off in
    the trainer: at C3 every GEMM fills the chip, and two side by side measured slower than in
    sequence (dWa beside dc: 67 + 67 us vs 37 + 37 us).
    """
    d, L = cfg.d, cfg.L
    B = a["B"]
    dev = gout.device
    st = _lib.stream_handle(dev)
    ntot = B if ntot is None else ntot
    KC = 15 * d
    scale = 1.0 / (1.0 - cfg.p_drop) if (cfg.training and cfg.p_drop > 0) else 1.0
    f32 = dict(dtype=torch.float32, device=dev)
    # head + BN2 backward (rank-1 source gout (x) Wc)
    bf = cfg.bf16
    w16 = a.get("w16")
    bf16_ = dict(dtype=torch.bfloat16, device=dev)
    lean = bf and coll.world <= 1             # f32 copies of dh2pre / dh1pre have no reader

    def tmp(name, shape, dtype=torch.float32):
        # the backward's scratch, kept in the activation dict: the native trainer's dict lives
        # across steps, so a step allocates nothing (host time); stream order keeps reuse safe
        t = a.get("bwd_" + name)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
            t = _lib.persistent(lambda: torch.empty(shape, dtype=dtype, device=dev))
            a["bwd_" + name] = t
        return t

    # bf16_fwd: the fp32 gradient GEMMs as split-bf16 x3 on the bf16 MFMA (fbn_gemm bf16 = 2;
    # FBN_SPLIT_BWD=0: fp32 MFMA)
    sb = 2 if (cfg.fwd16 and _SPLIT_BWD) else False
    # bf16_fwd: every backward GEMM as ONE bf16 GEMM over 3 K on (hi, lo) images of its fp32 operands
    # (split_images; fbn_gemm_s3 / split-bf16 x3 slabs) where the LDS-DMA path takes the shape, else
    # the fp32 MFMA
    s3 = cfg.fwd16 and _SPLIT3 and not bf and not cfg.bilinear_each
    # ... with every operand image made by its producing kernel (forward: fbn_pairs_fwd_img,
    # fbn_bn_act_fwd_img, the weight conversion; here: the BN backward, fbn_pairs_bwd_img): no fp32
    # dh2 / dh1 / dU and no conversion pass but dhmm's
    s3img = s3 and bool(a.get("s3img"))
    im = {}

    def img(name, rows, cols):
        return tmp("s3_" + name, (2, rows, cols), torch.bfloat16)

    if s3:
        # the operands the forward left and the weights: ONE launch (none when the forward made them)
        jobs = []
        for name, src, rows, cols, ld, trans, rm in (("WbT", p["mlp.4.weight"], H1, H2, H1, 1, NO_REMAP),
                                                     ("WaT", p["mlp.0.weight"], KC, H1, 21 * d, 1, wa_remap(d)),
                                                     ("W", p["bilinear.W"], d, d, d, 0, NO_REMAP),
                                                     ("x", batch["item_emb_d128"], B, 128, 128, 0, NO_REMAP)):
            t = a.get("s3w_" + name) if a.get("s3w") else None
            if t is not None and tuple(t.shape) == (2, rows, cols):
                im[name] = t                        # the forward's weight conversion wrote both images
            else:
                im[name] = img(name, rows, cols)
                jobs.append((src, im[name], rows, cols, ld, trans, rm))
        if s3img:
            im["h1"] = a["s3_h1"]                   # fbn_bn_act_fwd_img
        else:
            im["h1"] = img("h1", B, H1)
            jobs.append((a["h1"], im["h1"], B, H1, H1, 0, NO_REMAP))
        if a.get("s3img"):
            im["Vc"] = a["s3_vc"]                   # written by fbn_pairs_fwd_img
        else:
            im["Vc"] = img("Vc", 5 * B, d)
            jobs.append((a["Vc"], im["Vc"], 5 * B, d, d, 0, NO_REMAP))
        if a.get("s3_c") is not None and tuple(a["s3_c"].shape) == (2, B, KC):
            im["c"] = a["s3_c"]                     # made by the forward (its layer-1 GEMM reads the hi image)
        else:
            im["c"] = img("c", B, KC)
            jobs.append((a["c"], im["c"], B, KC, KC, 0, NO_REMAP))
        if jobs:
            split_images(jobs, st)
    dh2pre = None if (lean or s3img) else tmp("dh2pre", (B, H2))
    dh2 = img("dh2", B, H2) if s3 else None
    dh2pre16 = tmp("dh2pre16", (B, H2), torch.bfloat16) if bf else None
    sums = DeferredSums(a)
    wg = _SideWork(side, dev)
    bn_backward(None, gout, p["mlp.8.weight"], a["h2"], scale, a["h2pre"], a["mean2"], a["inv2"],
                p["mlp.5.weight"], B, H2, ntot, dh2pre, g["mlp.5.weight"], g["mlp.5.bias"], g["mlp.8.weight"],
                coll, st, dpre16=dh2pre16, bias_grad=g["mlp.4.bias"], sums=sums,
                part_pre=a.get("bn2_bwd_part") if (gout is a.get("gout")) else None, tag="bn2",
                dpre_img=dh2 if s3img else None)
    sums.add(gout, B, 1, g["mlp.8.bias"])
    dh1 = tmp("dh1", (B, H1))
    part1 = None
    lean_h1 = a.get("lean_h1", False)
    if bf:
        if not sums.gemm_slabs(dh2pre16, a["h1_16"], g["mlp.4.weight"], H2, H1, B, H2, H1, H1, True, False,
                               stream=st):
            wg.run(lambda s: gemm(dh2pre16, a["h1_16"], g["mlp.4.weight"], H2, H1, B, H2, H1, H1, True, False,
                                  stream=s))
        if (_BN1_BWD_IN_GEMM and lean_h1 and coll.world <= 1
                and _lib.lib().fbn_gemm_bn_bwd_part_supported(B, H1, H2, H2, H2, 0, 1)):
            # dh1 = dh2 Wb and, from its accumulators, the BN1 backward's column partials (no pass
            # over dh1 to compute them)
            part1 = tmp("part1", (_lib.lib().fbn_bn_bwd_chunks(B, H1) * 3 * H1,), torch.float64)
            call("fbn_gemm_bn_bwd_part", ptr(dh2pre16), ptr(w16["WbT"]), ptr(dh1), B, H1, H2, H2, H2, H1, 0, 1,
                 ptr(a["h1_16"]), ptr(a["h1pre"]), ptr(a["mean1"]), float(scale), ptr(part1), st)
        else:
            gemm(dh2pre16, w16["WbT"], dh1, B, H1, H2, H2, H2, H1, False, True, stream=st)
    elif s3:
        if not s3img:
            split_images([(dh2pre, dh2, B, H2, H2, 0, NO_REMAP)], st)
        if not sums.gemm_slabs(dh2, im["h1"], g["mlp.4.weight"], H2, H1, B, H2, H1, H1, True, False, stream=st,
                               s3=True):
            if s3_ok(H2, H1, B, H2, H1, True, False):
                wg.run(lambda s: gemm_s3(dh2, im["h1"], g["mlp.4.weight"], H2, H1, B, H2, H1, H1, True, False,
                                         stream=s))
            else:
                wg.run(lambda s: gemm(dh2pre, a["h1"], g["mlp.4.weight"], H2, H1, B, H2, H1, H1, True, False,
                                      stream=s))
        if s3_ok(B, H1, H2, H2, H2, False, True):
            gemm_s3(dh2, im["WbT"], dh1, B, H1, H2, H2, H2, H1, False, True, stream=st)
        else:
            gemm(dh2pre, p["mlp.4.weight"], dh1, B, H1, H2, H2, H1, H1, False, False, stream=st)
    else:
        wg.run(lambda s: gemm(dh2pre, a["h1"], g["mlp.4.weight"], H2, H1, B, H2, H1, H1, True, False, bf16=sb,
                              stream=s))
        gemm(dh2pre, p["mlp.4.weight"], dh1, B, H1, H2, H2, H1, H1, False, False, bf16=sb, stream=st)
    dh1pre = None if (lean or s3img) else tmp("dh1pre", (B, H1))
    dh1pre16 = tmp("dh1pre16", (B, H1), torch.bfloat16) if bf else None
    dh1i = img("dh1", B, H1) if s3 else None
    bn_backward(dh1, None, None, None if lean_h1 else a["h1"], scale, a["h1pre"], a["mean1"], a["inv1"],
                p["mlp.1.weight"], B, H1, ntot, dh1pre, g["mlp.1.weight"], g["mlp.1.bias"], None, coll, st,
                dpre16=dh1pre16, bias_grad=g["mlp.0.bias"], sums=sums, hact16=a["h1_16"] if lean_h1 else None,
                part_pre=part1, tag="bn1", dpre_img=dh1i if s3img else None)
    # weight gradient of the MLP input layer (side work), then its dgrad dc
    if s3:
        if not s3img:
            split_images([(dh1pre, dh1i, B, H1, H1, 0, NO_REMAP)], st)
        if not sums.gemm_slabs(dh1i, im["c"], g["mlp.0.weight"], H1, KC, B, H1, KC, 21 * d, True, False,
                               rC=wa_remap(d), stream=st, s3=True):
            wg.run(lambda s: gemm(dh1pre, a["c"], g["mlp.0.weight"], H1, KC, B, H1, KC, 21 * d, True, False,
                                  rC=wa_remap(d), stream=s))
    elif a.get("split_c"):
        if not sums.gemm_slabs(dh1pre16, a["Vc16"], g["mlp.0.weight"], H1, KC, B, H1, 5 * d, 21 * d, True, False,
                               rC=wa_remap(d), stream=st, B2=a["c"][:, 5 * d:], ldb2=KC, nseg=5 * d):
            wg.run(lambda s: gemm_split(dh1pre16, a["Vc16"], g["mlp.0.weight"], H1, KC, B, H1, 5 * d, 21 * d, True,
                                        False, rC=wa_remap(d), stream=s, B2=a["c"][:, 5 * d:], ldb2=KC, nseg=5 * d))
    elif bf:
        # (d < 128: the MLP input c is one bf16 operand) slabs in the step's grouped launch when the
        # shape allows, else a launch of its own with its split-K reduce
        ldcc = a["c"].shape[1]                      # wa_ld(d): c's rows carry zero columns past 15d
        if not sums.gemm_slabs(dh1pre16, a["c"], g["mlp.0.weight"], H1, KC, B, H1, ldcc, 21 * d, True, False,
                               rC=wa_remap(d), stream=st):
            wg.run(lambda s: gemm(dh1pre16, a["c"], g["mlp.0.weight"], H1, KC, B, H1, ldcc, 21 * d, True, False,
                                  rC=wa_remap(d), stream=s))
    else:
        wg.run(lambda s: gemm(dh1pre, a["c"], g["mlp.0.weight"], H1, KC, B, H1, KC, 21 * d, True, False,
                              rC=wa_remap(d), bf16=sb, stream=s))
    if a.get("fused_bilinear"):
        # dc in bf16: its one reader, the fused bilinear backward, widens it on load
        dc = tmp("dc16", (B, KC), torch.bfloat16)
        call("fbn_gemm_bf16out", ptr(dh1pre16), ptr(w16["WaT"]), ptr(dc), B, KC, H1, H1, H1, KC, 0, 1, st)
    elif bf:
        dc = torch.empty((B, KC), **f32)
        gemm(dh1pre16, w16["WaT"], dc, B, KC, H1, H1, H1, KC, False, True, stream=st)
    elif s3 and s3_ok(B, KC, H1, H1, H1, False, True):
        dc = torch.empty((B, KC), **f32)
        gemm_s3(dh1i, im["WaT"], dc, B, KC, H1, H1, H1, KC, False, True, stream=st)
    else:
        dc = torch.empty((B, KC), **f32)
        gemm(dh1pre, p["mlp.0.weight"], dc, B, KC, H1, H1, 21 * d, KC, False, False, rB=wa_remap(d), bf16=sb,
             stream=st)
    # bilinear backward
    dV = tmp("dV", (B, 5, d))
    v16 = bf and not cfg.bilinear_each
    dU16 = tmp("dU16", (B, 5, d), torch.bfloat16) if v16 else None
    if a.get("fused_bilinear"):
        # one launch: dU and dV = dc_V + pair terms + dU W^T (U recomputed on the MFMA)
        call("fbn_bilinear_bwd", ptr(dc), KC, int(dc.dtype == torch.bfloat16), ptr(a["Vc16"]), ptr(w16["WT"]),
             ptr(w16["W"]), ptr(dV), ptr(dU16), B, d, st)
        if not sums.gemm_slabs(a["Vc16"], dU16, g["bilinear.W"], d, d, 5 * B, d, d, d, True, False, stream=st):
            wg.run(lambda s: gemm(a["Vc16"], dU16, g["bilinear.W"], d, d, 5 * B, d, d, d, True, False, stream=s))
    elif s3 and a.get("s3img"):
        dU = None                                   # only its split images (every reader takes them)
        dU2 = img("dU", 5 * B, d)
        call("fbn_pairs_bwd_img", ptr(dc), ptr(a["Vc"]), ptr(a["U"]), ptr(dV), ptr(dU2), B, d, KC, st)
    else:
        dU = torch.empty((B, 5, d), **f32)
        call("fbn_pairs_bwd", ptr(dc), None if v16 else ptr(a["Vc"]), ptr(a["Vc16"]) if v16 else None, ptr(a["U"]),
             ptr(dV), ptr(dU), ptr(dU16), B, d, KC, int(cfg.bilinear_each), st)
    if a.get("fused_bilinear"):
        pass
    elif not cfg.bilinear_each:
        if bf:
            if not sums.gemm_slabs(a["Vc16"], dU16, g["bilinear.W"], d, d, 5 * B, d, d, d, True, False, stream=st):
                wg.run(lambda s: gemm(a["Vc16"], dU16, g["bilinear.W"], d, d, 5 * B, d, d, d, True, False, stream=s))
            gemm(dU16, w16["W"], dV, 5 * B, d, d, d, d, d, False, True, beta=1.0, stream=st)
        elif s3:
            if dU is not None:
                dU2 = img("dU", 5 * B, d)
                split_images([(dU, dU2, 5 * B, d, d, 0, NO_REMAP)], st)
            if not sums.gemm_slabs(im["Vc"], dU2, g["bilinear.W"], d, d, 5 * B, d, d, d, True, False, stream=st,
                                   s3=True):
                wg.run(lambda s: gemm(a["Vc"], dU, g["bilinear.W"], d, d, 5 * B, d, d, d, True, False, stream=s))
            if s3_ok(5 * B, d, d, d, d, False, True):
                gemm_s3(dU2, im["W"], dV, 5 * B, d, d, d, d, d, False, True, beta=1.0, stream=st)
            else:
                gemm(dU, p["bilinear.W"], dV, 5 * B, d, d, d, d, d, False, True, beta=1.0, stream=st)
        else:
            wg.run(lambda s: gemm(a["Vc"], dU, g["bilinear.W"], d, d, 5 * B, d, d, d, True, False, bf16=sb,
                                  stream=s))
            gemm(dU, p["bilinear.W"], dV, 5 * B, d, d, d, d, d, False, True, beta=1.0, bf16=sb, stream=st)
    else:
        g["bilinear.W_list.0"].zero_()
        for f in range(1, 5):
            gemm(dU[:, f - 1], p[f"bilinear.W_list.{f}"], dV[:, f - 1], B, d, d, 5 * d, d, 5 * d, False, True,
                 beta=1.0, bf16=cfg.bf16, stream=st)
            gemm(a["Vc"][:, f - 1], dU[:, f - 1], g[f"bilinear.W_list.{f}"], d, d, B, 5 * d, 5 * d, d, True, False,
                 bf16=cfg.bf16, stream=st)
    if hooks and "after_bilinear_bwd" in hooks:   # trainer: the weight gradients so far launched early
        hooks["after_bilinear_bwd"](sums)
    # fields backward: SENET, LN, cate + item-table scatter
    R = cfg.R
    ncate = p["cate_emb.weight"].shape[0]
    P = _lib.lib().fbn_fields_bwd_partials_size(d, R, ncate)
    nblk = _lib.lib().fbn_fields_bwd_grid(B, d)
    partials = tmp("partials", (nblk, P))
    dhmm = tmp("dhmm", (B, d))
    dhmm16 = tmp("dhmm16", (B, d), torch.bfloat16) if bf else None
    dhs = img("dhmm", B, d) if s3 else None
    seq = batch.get("item_seq", None)
    Lr = 0 if seq is None else L
    V = p["item_emb.weight"].shape[0] if pos is None else 0
    keys = ("senet.excitation.0.weight", "senet.excitation.0.bias", "senet.excitation.2.weight",
            "senet.excitation.2.bias", "mm_proj.1.weight", "mm_proj.1.bias", "cate_emb.weight", "mm_proj.0.bias")
    if _DEFER_REDUCE:
        outs = None       # the partial rows' segments are summed in the step's sum_jobs launch
        o = 0
        for k, n in zip(keys, (6 * R, R, 6 * R, 6, d, d, ncate * d, d)):
            sums.add(partials[:, o:], nblk, n, g[k], ld=P)
            o += n
    else:
        outs_arr = (ctypes.c_void_p * 8)(*[g[k].data_ptr() for k in keys])   # host array of device pointers
        _lib.keep(outs_arr)
        outs = ctypes.cast(outs_arr, ctypes.c_void_p).value
    evb = _probe_start(probe, "fields_bwd")     # bench / tools: the fields backward
    call("fbn_fields_bwd_img" if s3img else "fbn_fields_bwd", ptr(batch["item_id"]), ptr(seq) if Lr else None,
         ptr(batch["likes_level"]),
         ptr(batch["views_level"]), ptr(a["hmm"]), ptr(p["mm_proj.1.weight"]), ptr(p["mm_proj.1.bias"]), LN_EPS,
         ptr(p["senet.excitation.0.weight"]), ptr(p["senet.excitation.0.bias"]), ptr(p["senet.excitation.2.weight"]),
         R, ncate, ptr(p["cate_emb.weight"]), ptr(a["X"]), ptr(a["a"]), ptr(a["cnt"]), ptr(dV), ptr(dhmm),
         ptr(dhs if s3img else dhmm16), ptr(partials), outs,
         ptr(table_grad), ptr(gvec), ptr(gnorm), V, ptr(pos), ptr(sendbuf),
         int(sendbuf is not None and sendbuf.dtype == torch.bfloat16), B, Lr, d, st)
    _probe_end(evb)
    if hooks and "after_fields_bwd" in hooks:     # N > 1: the gradient rows are complete -> exchange
        hooks["after_fields_bwd"]()
    if bf:
        if not sums.gemm_slabs(dhmm16, w16["x"], g["mm_proj.0.weight"], d, 128, B, d, 128, 128, True, False,
                               stream=st):
            wg.run(lambda s: gemm(dhmm16, w16["x"], g["mm_proj.0.weight"], d, 128, B, d, 128, 128, True, False,
                                  stream=s))
    elif s3:
        if not s3img:
            split_images([(dhmm, dhs, B, d, d, 0, NO_REMAP)], st)
        if not sums.gemm_slabs(dhs, im["x"], g["mm_proj.0.weight"], d, 128, B, d, 128, 128, True, False,
                               stream=st, s3=True):
            wg.run(lambda s: gemm(dhmm, batch["item_emb_d128"], g["mm_proj.0.weight"], d, 128, B, d, 128, 128, True,
                                  False, stream=s))
    else:
        wg.run(lambda s: gemm(dhmm, batch["item_emb_d128"], g["mm_proj.0.weight"], d, 128, B, d, 128, 128, True,
                              False, bf16=sb, stream=s))
    for job in extra_sums:              # e.g. the trainer's mean loss
        sums.add(*job)
    if hooks and "before_flush" in hooks:         # trainer: join the early weight-gradient launch
        hooks["before_flush"]()
    sums.flush(st, probe)
    wg.join()
