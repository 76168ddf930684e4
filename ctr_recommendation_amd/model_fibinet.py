"""Drop-in replacement for the reference ``src/model_fibinet.py`` on MI355X.

Same public surface as the reference module:

* ``build_model(feature_map, model_cfg) -> nn.Module``                 (model_fibinet.py:201-202)
* ``MM_FiBiNET(feature_map, model_cfg)`` with ``forward(batch_dict) -> probs[B]`` (:91-199)
* ``SENetLayer(num_fields, reduction_ratio)`` / ``BilinearInteraction(input_dim, num_fields,
  bilinear_type)`` as parameter containers with the reference names (:5-89)
* identical parameter creation order (seeded inits match the reference bit for bit) and the
  exact App. B ``state_dict`` keys/shapes, so checkpoints interchange both ways;
* ``ValueError`` for an unknown ``bilinear_type`` (:57-58).

Every forward/backward FLOP runs in libfibinet_hip.so (ops.py sequences the kernels); a
tensor that is not on a HIP device raises -- there is no CPU fallback.  The backward fills a
dense ``item_emb.weight.grad`` (V x d) exactly as ``nn.Embedding`` does, so the unchanged
reference ``train_fibinet.py`` (torch Adam, clip_grad_norm_) drives it as-is.

Opt-in extensions the reference's config names but its code ignores (off unless
``honour_config: true`` is set in model_cfg): ``vocab_size``, ``bilinear_type``,
``senet_reduction``, ``net_dropout``.  ``compute_dtype: bf16`` runs every GEMM with bf16
operands and fp32 accumulation; ``compute_dtype: bf16_fwd`` only the forward GEMMs, the backward
in fp32 (config C3's "bf16 fwd / fp32 grad accum").
"""
from __future__ import annotations

import functools
from typing import Dict, List, Tuple

import torch
import torch.nn as nn

from . import _lib, ops

NUM_FIELDS = 6
MM_INPUT_DIM = 128
REFERENCE_VOCAB = 91718
USER_VOCAB = 20000
CATE_VOCAB = 11


class SENetLayer(nn.Module):
    """Squeeze-excitation parameters (model_fibinet.py:5-22); computed by fields.hip."""

    def __init__(self, num_fields, reduction_ratio=3):
        super().__init__()
        reduced = max(1, num_fields // reduction_ratio)
        self.excitation = nn.Sequential(nn.Linear(num_fields, reduced), nn.ReLU(),
                                        nn.Linear(reduced, num_fields), nn.Sigmoid())


class BilinearInteraction(nn.Module):
    """Bilinear-interaction parameters (model_fibinet.py:37-58); computed by gemm.hip + mlp.hip."""

    def __init__(self, input_dim, num_fields, bilinear_type="all"):
        super().__init__()
        self.bilinear_type = bilinear_type
        if bilinear_type == "all":
            self.W = nn.Parameter(torch.Tensor(input_dim, input_dim))
            nn.init.xavier_normal_(self.W)
        elif bilinear_type == "each":
            self.W_list = nn.ParameterList(
                [nn.Parameter(torch.Tensor(input_dim, input_dim)) for _ in range(num_fields - 1)])
            for w in self.W_list:
                nn.init.xavier_normal_(w)
        else:
            raise ValueError("bilinear_type must be 'all' or 'each'")


class _FiBiNETFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, module, batch, *params):
        names = module._param_names
        p = dict(zip(names, params))
        p.update(module._buffers_dict())
        cfg = module._fwd_cfg()
        if "item_seq" in batch:
            cfg.L = batch["item_seq"].shape[1]
        rng = module._rng_state(batch["item_id"].device) if cfg.training and cfg.p_drop > 0 else None
        acts = ops.forward(p, batch, cfg, rng)
        module._check_ids(acts["err"])
        if rng is not None:
            rng[1] += 1
        ctx.module = module
        ctx.cfg = cfg
        ctx.batch = batch
        ctx.acts = acts
        ctx.p = p
        ctx.save_for_backward(acts["probs"])
        return acts["probs"].clone()

    @staticmethod
    def backward(ctx, grad_probs):
        (probs,) = ctx.saved_tensors
        module, p, a, cfg = ctx.module, ctx.p, ctx.acts, ctx.cfg
        B = probs.shape[0]
        dev = probs.device
        st = _lib.stream_handle(dev)
        gout = torch.empty(B, dtype=torch.float32, device=dev)
        _lib.call("fbn_sigmoid_bwd", _lib.ptr(grad_probs.contiguous().float()), _lib.ptr(probs), _lib.ptr(gout), B, st)
        g = {n: torch.empty_like(p[n]) for n in module._param_names}
        g["mlp.0.weight"].zero_()            # the 6d structurally-zero input columns get exactly 0
        table_grad = torch.zeros_like(p["item_emb.weight"])
        ops.backward(p, ctx.batch, a, gout, g, cfg, table_grad=table_grad)
        g["item_emb.weight"] = table_grad
        grads: List = [None, None]
        for n in module._param_names:
            grads.append(None if n == "user_emb.weight" else g.get(n))
        return tuple(grads)


class MM_FiBiNET(nn.Module):
    """MI355X-native MM-FiBiNET with the reference's constructor, forward and state_dict."""

    def __init__(self, feature_map, model_cfg):
        super().__init__()
        self.emb_dim = model_cfg.get("embedding_dim", 64)
        honour = bool(model_cfg.get("honour_config", False))
        vocab = int(model_cfg.get("vocab_size", REFERENCE_VOCAB))   # extension key; reference: 91718
        btype = model_cfg.get("bilinear_type", "all") if honour else "all"
        red = int(model_cfg.get("senet_reduction", 2)) if honour else 2
        self.dropout_p = float(model_cfg.get("net_dropout", 0.2)) if honour else 0.2
        cdt = str(model_cfg.get("compute_dtype", "fp32")).lower()
        if cdt not in ("fp32", "float32", "bf16", "bfloat16", "bf16_fwd"):
            raise ValueError(f"compute_dtype must be 'fp32', 'bf16' or 'bf16_fwd', not {cdt!r}")
        # bf16: every GEMM operand bf16 (forward and backward); bf16_fwd: the forward GEMMs take bf16
        # operands, the backward runs in fp32 from fp32 activations (C3's "bf16 fwd / fp32 grad")
        self.compute_bf16 = cdt in ("bf16", "bfloat16")
        self.compute_fwd16 = cdt == "bf16_fwd"
        d = self.emb_dim
        # creation order == reference (:100-136)
        self.item_emb = nn.Embedding(vocab, d, padding_idx=0)
        self.user_emb = nn.Embedding(USER_VOCAB, d)
        self.cate_emb = nn.Embedding(CATE_VOCAB, d)
        self.mm_proj = nn.Sequential(nn.Linear(MM_INPUT_DIM, d), nn.LayerNorm(d), nn.ReLU())
        self.num_fields = NUM_FIELDS
        self.senet = SENetLayer(self.num_fields, reduction_ratio=red)
        self.bilinear = BilinearInteraction(d, self.num_fields, bilinear_type=btype)
        num_pairs = (self.num_fields * (self.num_fields - 1)) // 2
        total_input_dim = (self.num_fields + num_pairs) * d
        self.mlp = nn.Sequential(
            nn.Linear(total_input_dim, 512), nn.BatchNorm1d(512), nn.ReLU(), nn.Dropout(self.dropout_p),
            nn.Linear(512, 256), nn.BatchNorm1d(256), nn.ReLU(), nn.Dropout(self.dropout_p),
            nn.Linear(256, 1))
        self.sigmoid = nn.Sigmoid()
        self._param_names = [n for n, _ in self.named_parameters()]
        # dropout streams, one per device.  The dict object is shared by nn.DataParallel replicas
        # (replicate() copies __dict__ shallowly), so each device's counter advances across steps
        # although the replicas themselves are rebuilt every forward (train_fibinet.py:69-70)
        self._rngs: Dict[int, torch.Tensor] = {}
        self._strict_ids = True

    # ---------------------------------------------------------------- helpers
    def _buffers_dict(self) -> Dict[str, torch.Tensor]:
        return {n: b for n, b in self.named_buffers()}     # replicas keep their buffers registered

    def _fwd_cfg(self) -> ops.FwdConfig:
        return ops.FwdConfig(d=self.emb_dim, L=0, training=self.training, p_drop=self.dropout_p,
                             bf16=self.compute_bf16, fwd16=self.compute_fwd16,
                             bilinear_each=self.bilinear.bilinear_type == "each",
                             R=self.senet.excitation[0].out_features)

    def _rng_state(self, device) -> torch.Tensor:
        idx = device.index if device.index is not None else torch.cuda.current_device()
        rng = self._rngs.get(idx)
        if rng is None:
            # does not advance torch's RNG stream; an independent stream per device
            seed = (torch.initial_seed() + idx * 0x9E3779B9) & 0xFFFFFFFFFFFF
            rng = torch.tensor([seed, 0], dtype=torch.int64, device=device)
            self._rngs[idx] = rng
        return rng

    def _param_tensors(self) -> List[torch.Tensor]:
        """The parameters in ``_param_names`` order, resolved by attribute.  On an nn.DataParallel
        replica ``named_parameters()`` is empty: replicate() sets the broadcast copies as plain
        attributes (non-leaf tensors whose grads flow back to the originals), which this finds."""
        out = []
        for n in self._param_names:
            t = functools.reduce(getattr, n.split("."), self)
            out.append(t if t.is_contiguous() else t.contiguous())
        return out

    def _check_ids(self, err: torch.Tensor) -> None:
        # the reference raises IndexError on an out-of-range id (nn.Embedding); the kernels set a
        # sticky device flag, checked here (one 4-byte read)
        if self._strict_ids and int(err.item()) != 0:
            raise IndexError("index out of range in self (item/likes/views id outside its embedding table)")

    # ---------------------------------------------------------------- forward
    def forward(self, batch_dict):
        item_id = batch_dict["item_id"]
        _lib.require_hip(item_id, "batch_dict['item_id']")
        _lib.require_hip(self.item_emb.weight, "model parameters")
        batch = {
            "item_id": item_id.long().contiguous(),
            "item_emb_d128": batch_dict["item_emb_d128"].float().contiguous(),
            "likes_level": batch_dict["likes_level"].long().contiguous(),
            "views_level": batch_dict["views_level"].long().contiguous(),
        }
        seq = batch_dict.get("item_seq", None)
        if seq is not None:
            batch["item_seq"] = seq.long().contiguous()
        return _FiBiNETFn.apply(self, batch, *self._param_tensors())


def build_model(feature_map, model_cfg):
    return MM_FiBiNET(feature_map, model_cfg)
