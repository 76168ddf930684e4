"""CPU restatement of MM-FiBiNET (forward, backward via autograd, train step).

TEST INFRASTRUCTURE ONLY -- see ``oracle/__init__.py``.  Imported by tests/, smoke() and
bench.py's cpu_baseline leg; never by the product package.

Every block cites the reference line it restates (paths relative to the reference root):

* parameters and their init order ........ src/model_fibinet.py:95-136
* field construction .................... src/model_fibinet.py:138-182
* SENET .................................. src/model_fibinet.py:5-35  (reduction 2 -> 6->3->6)
* bilinear "all" (W on the 2nd field) .... src/model_fibinet.py:60-79, 89
* bilinear "each" (dead in the reference,
  kept for the opt-in config surface) .... src/model_fibinet.py:50-56, 81-86
* concat + MLP + sigmoid ................. src/model_fibinet.py:191-199
* train step ............................. src/train_fibinet.py:78-92, 113-124
* AUC / logloss .......................... src/utils.py:18-32

The module keeps the reference's submodule names so ``state_dict()`` has exactly the App. B
keys.  Parameter creation order is the reference's, so a seeded
construction draws the same initial weights.  ``forward`` optionally takes explicit dropout
masks so the HIP path (which uses its own counter-based RNG) can be compared bit-for-mask.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

NUM_FIELDS = 6            # [user, likes, views, item, image, history]  model_fibinet.py:112-113
MM_INPUT_DIM = 128        # model_fibinet.py:96
REFERENCE_VOCAB = 91718   # model_fibinet.py:100 (hard-coded)
USER_VOCAB = 20000        # model_fibinet.py:101
CATE_VOCAB = 11           # model_fibinet.py:102
DROPOUT_P = 0.2           # model_fibinet.py:129,133 (hard-coded; config's net_dropout is dead)
HIDDEN = (512, 256)       # model_fibinet.py:126,130


def pair_list(num_fields: int = NUM_FIELDS) -> Sequence[Tuple[int, int]]:
    """Lexicographic i<j pairs, the order of model_fibinet.py:75-79."""
    return [(i, j) for i in range(num_fields) for j in range(i + 1, num_fields)]


class _SENet(nn.Module):
    # model_fibinet.py:10-22: reduced = max(1, F // ratio); Linear, ReLU, Linear, Sigmoid
    def __init__(self, num_fields: int, reduction_ratio: int):
        super().__init__()
        reduced = max(1, num_fields // reduction_ratio)
        self.excitation = nn.Sequential(
            nn.Linear(num_fields, reduced), nn.ReLU(), nn.Linear(reduced, num_fields), nn.Sigmoid())

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        z = x.mean(dim=-1)                       # squeeze over the embedding dim (:28)
        a = self.excitation(z)                   # (:31)
        return x * a.unsqueeze(-1)               # (:35)


class _Bilinear(nn.Module):
    def __init__(self, d: int, num_fields: int, bilinear_type: str):
        super().__init__()
        self.bilinear_type = bilinear_type
        if bilinear_type == "all":
            self.W = nn.Parameter(torch.empty(d, d))
            nn.init.xavier_normal_(self.W)
        elif bilinear_type == "each":
            self.W_list = nn.ParameterList([nn.Parameter(torch.empty(d, d)) for _ in range(num_fields - 1)])
            for w in self.W_list:
                nn.init.xavier_normal_(w)
        else:  # model_fibinet.py:57-58
            raise ValueError("bilinear_type must be 'all' or 'each'")

    def forward(self, v: torch.Tensor) -> torch.Tensor:
        nf = v.shape[1]
        out = []
        if self.bilinear_type == "all":
            u = torch.matmul(v, self.W)          # W applied to every field; used on field j (:72,79)
            for i, j in pair_list(nf):
                out.append(v[:, i, :] * u[:, j, :])
        else:
            for i, j in pair_list(nf):           # W_i applied to field i (:85-86)
                out.append(torch.matmul(v[:, i, :], self.W_list[i]) * v[:, j, :])
        return torch.stack(out, dim=1)


class OracleFiBiNET(nn.Module):
    """Restatement of ``MM_FiBiNET`` (model_fibinet.py:91-199).

    ``model_cfg`` keys read: ``embedding_dim`` (default 64, :95).  Opt-in keys that the
    reference ignores (defaults reproduce the reference exactly): ``vocab_size``
    (default 91718), ``bilinear_type`` (default "all"), ``senet_reduction`` (default 2),
    ``net_dropout`` (default 0.2).  The opt-in keys are only honoured when
    ``honour_config=True`` so that the reference config (which says "each", 0.25) still
    builds the code's model.
    """

    def __init__(self, model_cfg: Dict, honour_config: bool = False):
        super().__init__()
        d = int(model_cfg.get("embedding_dim", 64))
        self.emb_dim = d
        vocab = int(model_cfg.get("vocab_size", REFERENCE_VOCAB))
        btype, red, p = "all", 2, DROPOUT_P
        if honour_config:
            btype = model_cfg.get("bilinear_type", btype)
            red = int(model_cfg.get("senet_reduction", red))
            p = float(model_cfg.get("net_dropout", p))
        self.dropout_p = p
        # creation order == reference order (:100-136) so seeded inits match
        self.item_emb = nn.Embedding(vocab, d, padding_idx=0)
        self.user_emb = nn.Embedding(USER_VOCAB, d)
        self.cate_emb = nn.Embedding(CATE_VOCAB, d)
        self.mm_proj = nn.Sequential(nn.Linear(MM_INPUT_DIM, d), nn.LayerNorm(d), nn.ReLU())
        self.num_fields = NUM_FIELDS
        self.senet = _SENet(NUM_FIELDS, red)
        self.bilinear = _Bilinear(d, NUM_FIELDS, btype)
        n_pairs = NUM_FIELDS * (NUM_FIELDS - 1) // 2
        din = (NUM_FIELDS + n_pairs) * d
        h1, h2 = HIDDEN
        self.mlp = nn.Sequential(
            nn.Linear(din, h1), nn.BatchNorm1d(h1), nn.ReLU(), nn.Dropout(p),
            nn.Linear(h1, h2), nn.BatchNorm1d(h2), nn.ReLU(), nn.Dropout(p),
            nn.Linear(h2, 1))
        self.sigmoid = nn.Sigmoid()

    # ------------------------------------------------------------------ fields
    def fields(self, batch: Dict[str, torch.Tensor]) -> torch.Tensor:
        """X = [0, C[likes], C[views], E[item], mm(x), masked-mean E[seq]]  (:140-182)."""
        item_id = batch["item_id"].long()
        # .float() in the reference (:141); a float64 copy of the oracle (tests' arbiter) keeps f64
        ft = self.item_emb.weight.dtype
        x_mm = batch["item_emb_d128"].to(ft)
        likes = batch["likes_level"].long()
        views = batch["views_level"].long()
        seq = batch.get("item_seq", None)
        b = item_id.shape[0]
        user = torch.zeros((b, self.emb_dim), device=item_id.device, dtype=ft)
        f_like = self.cate_emb(likes)
        f_view = self.cate_emb(views)
        f_item = self.item_emb(item_id)
        f_img = self.mm_proj(x_mm)
        if seq is not None:
            seq = seq.long()
            keep = (seq != 0)
            rows = self.item_emb(seq) * keep.unsqueeze(-1).to(ft)
            cnt = keep.to(ft).sum(dim=1, keepdim=True).clamp(min=1)
            f_hist = rows.sum(dim=1) / cnt
        else:
            f_hist = torch.zeros_like(f_item)
        return torch.stack([user, f_like, f_view, f_item, f_img, f_hist], dim=1)

    def forward(self, batch: Dict[str, torch.Tensor],
                masks: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                return_logits: bool = False) -> torch.Tensor:
        x = self.fields(batch)
        v = self.senet(x)
        pairs = self.bilinear(v)
        b = x.shape[0]
        c = torch.cat([v.reshape(b, -1), pairs.reshape(b, -1)], dim=1)
        lin1, bn1, _, drop1, lin2, bn2, _, drop2, lin3 = self.mlp
        h = torch.relu(bn1(lin1(c)))
        h = self._drop(h, drop1, None if masks is None else masks[0])
        h = torch.relu(bn2(lin2(h)))
        h = self._drop(h, drop2, None if masks is None else masks[1])
        logits = lin3(h)
        if return_logits:
            return logits.squeeze(-1)
        return self.sigmoid(logits).squeeze(-1)

    def _drop(self, h, module, mask):
        if not self.training or self.dropout_p == 0.0:
            return h
        if mask is None:
            return module(h)                       # torch RNG (used by the known-answer test)
        # injected keep-mask; torch scales kept units by 1/(1-p) (ATen dropout)
        return h * (mask.to(h.dtype) * (1.0 / (1.0 - self.dropout_p)))


def build_model(feature_map, model_cfg, honour_config: bool = False) -> OracleFiBiNET:
    """Mirror of ``build_model`` (model_fibinet.py:201-202); feature_map is ignored."""
    return OracleFiBiNET(model_cfg, honour_config=honour_config)


# ---------------------------------------------------------------------- train step
class OracleTrainer:
    """The per-step part of train_fibinet.py:78-124 on CPU.

    Adam(lr, weight_decay) with coupled L2 (:78), BCELoss (:79), OneCycleLR(max_lr=10*lr,
    pct_start=0.3, div 25, final_div 1000, cos, beta1 cycled 0.95<->0.85) (:84-92),
    zero_grad -> fwd -> BCE -> bwd -> clip_grad_norm_(10) -> step -> sched.step (:113-123).

    Opt-in variants the build offers (non-parity with the reference's code, which uses Adam):
    optimizer="adamw" -> torch.optim.AdamW (the config's dead ``optimizer: adamw``,
    config/fibinet_config.yaml:62); table_optimizer="sparse" -> item_emb.weight is updated only
    on the rows the batch touches (torch.optim.SparseAdam's rule: moments and weights of the other
    rows stay as they are; bias corrections of the global step), with the optimizer's weight-decay
    rule applied to those rows.
    """

    def __init__(self, model: OracleFiBiNET, lr: float = 1e-3, weight_decay: float = 1e-5,
                 total_steps: int = 1000, max_norm: float = 10.0, optimizer: str = "adam",
                 table_optimizer: str = "dense"):
        self.model = model
        self.max_norm = max_norm            # train_fibinet.py:119 uses 10.0; tests lower it to engage the clip
        self.last_total_norm = None
        self.sparse_table = table_optimizer == "sparse"
        self.decoupled = optimizer == "adamw"
        params = [p for n, p in model.named_parameters() if not (self.sparse_table and n == "item_emb.weight")]
        cls = torch.optim.AdamW if self.decoupled else torch.optim.Adam
        self.opt = cls(params, lr=lr, weight_decay=weight_decay)
        self.loss_fn = nn.BCELoss()
        self.sched = torch.optim.lr_scheduler.OneCycleLR(
            self.opt, max_lr=lr * 10, total_steps=total_steps, pct_start=0.3,
            div_factor=25.0, final_div_factor=1000.0)
        self.t = 0
        if self.sparse_table:
            E = model.item_emb.weight
            self.Em, self.Ev = torch.zeros_like(E), torch.zeros_like(E)

    def _sparse_table_step(self, batch) -> None:
        E = self.model.item_emb.weight
        ids = [batch["item_id"].long().flatten()]
        if "item_seq" in batch:
            ids.append(batch["item_seq"].long().flatten())
        rows = torch.unique(torch.cat(ids))
        rows = rows[rows != 0]                                 # padding_idx=0 never receives a gradient
        grp = self.opt.param_groups[0]
        lr, (b1, b2), wd, eps = grp["lr"], grp["betas"], grp["weight_decay"], grp["eps"]
        t = self.t
        with torch.no_grad():
            p = E[rows]
            g = E.grad[rows]
            if self.decoupled:
                p = p * (1 - lr * wd)
            else:
                g = g + wd * p
            m = self.Em[rows].lerp(g, 1 - b1)
            v = self.Ev[rows] * b2 + (1 - b2) * g * g
            bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
            p = p + (-lr / bc1) * m / (v.sqrt() / math.sqrt(bc2) + eps)
            E[rows] = p
            self.Em[rows] = m
            self.Ev[rows] = v

    def _replicated_forward(self, batch, replicas: int) -> torch.Tensor:
        """nn.DataParallel's forward over `replicas` devices (train_fibinet.py:69-70): the batch is
        scattered in equal contiguous slices, each replica's BatchNorm1d normalises its own slice,
        the outputs are gathered in order; running statistics (and num_batches_tracked) keep
        only the device-0 replica's update -- the other replicas update broadcast copies."""
        n = next(iter(batch.values())).shape[0]
        per = n // replicas
        bns = [mod for mod in self.model.modules() if isinstance(mod, nn.BatchNorm1d)]
        keep = [(mod, dict(mod._buffers)) for mod in bns]
        outs = [None] * replicas
        for r in range(1, replicas):
            for mod, b in keep:                 # a replica's own copies (autograd keeps them)
                for name, t in b.items():
                    setattr(mod, name, t.clone())
            outs[r] = self.model({k: v[r * per:(r + 1) * per] for k, v in batch.items()})
        for mod, b in keep:
            for name, t in b.items():
                setattr(mod, name, t)
        outs[0] = self.model({k: v[:per] for k, v in batch.items()})
        return torch.cat(outs)

    def step(self, batch, labels, masks=None, replicas: int = 1) -> Tuple[float, torch.Tensor]:
        self.model.train()
        self.opt.zero_grad()
        if self.sparse_table:
            self.model.item_emb.weight.grad = None
        if replicas > 1:
            y = self._replicated_forward(batch, replicas)
        else:
            y = self.model(batch, masks=masks)
        loss = self.loss_fn(y, labels)
        loss.backward()
        self.last_total_norm = float(torch.nn.utils.clip_grad_norm_(self.model.parameters(), max_norm=self.max_norm))
        self.t += 1
        if self.sparse_table:
            self._sparse_table_step(batch)
        self.opt.step()
        self.sched.step()
        return float(loss.item()), y.detach()


# ---------------------------------------------------------------------- metrics
def compute_auc(y_true: np.ndarray, y_pred: np.ndarray) -> float:
    """ROC-AUC with average ranks for ties; 0.5 for single-class input (utils.py:18-27).

    Rank-sum (Mann-Whitney) form of sklearn's roc_auc_score; cross-checked against
    sklearn in tests/test_oracle.py.
    """
    y_true = np.asarray(y_true).astype(np.float64).ravel()
    y_pred = np.asarray(y_pred).astype(np.float64).ravel()
    pos = y_true == 1
    n_pos = int(pos.sum())
    n_neg = y_true.size - n_pos
    if n_pos == 0 or n_neg == 0:
        return 0.5
    order = np.argsort(y_pred, kind="mergesort")
    s = y_pred[order]
    ranks = np.empty(s.size, dtype=np.float64)
    i = 0
    while i < s.size:
        j = i
        while j + 1 < s.size and s[j + 1] == s[i]:
            j += 1
        ranks[i:j + 1] = 0.5 * (i + j) + 1.0
        i = j + 1
    r = np.empty_like(ranks)
    r[order] = ranks
    return float((r[pos].sum() - n_pos * (n_pos + 1) / 2.0) / (n_pos * n_neg))


def compute_logloss(y_true: np.ndarray, y_pred: np.ndarray, eps: float = 1e-15) -> float:
    """utils.py:29-32 (sklearn log_loss with labels=[0,1]); clipped at eps."""
    y = np.asarray(y_true, dtype=np.float64).ravel()
    p = np.clip(np.asarray(y_pred, dtype=np.float64).ravel(), eps, 1 - eps)
    return float(-np.mean(y * np.log(p) + (1 - y) * np.log(1 - p)))


def one_cycle_lr_beta1(step: int, total_steps: int, base_lr: float = 1e-3,
                       pct_start: float = 0.3, div_factor: float = 25.0,
                       final_div_factor: float = 1000.0,
                       max_momentum: float = 0.95, base_momentum: float = 0.85):
    """(lr, beta1) that OneCycleLR sets for optimizer step ``step`` (0-based); scalar restatement
    used to cross-check the product's host schedule against the Kaggle log."""
    max_lr = base_lr * 10
    initial = max_lr / div_factor
    min_lr = initial / final_div_factor
    end1 = float(pct_start * total_steps) - 1
    end2 = total_steps - 1
    if step <= end1:
        pct = step / end1
        lo, hi, mlo, mhi = initial, max_lr, max_momentum, base_momentum
    else:
        pct = (step - end1) / (end2 - end1)
        lo, hi, mlo, mhi = max_lr, min_lr, base_momentum, max_momentum
    cosf = lambda a, b, p: b + (a - b) / 2.0 * (math.cos(math.pi * p) + 1)
    return cosf(lo, hi, pct), cosf(mlo, mhi, pct)
