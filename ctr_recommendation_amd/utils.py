"""set_seed / compute_auc / compute_logloss with the semantics of the reference src/utils.py.

compute_auc (utils.py:18-27): ROC-AUC with ties at average rank (sklearn roc_auc_score) and
0.5 when the labels hold a single class.  Computed here as the Mann-Whitney rank-sum in
float64 (O(n log n), no sklearn dependency); tests cross-check it against sklearn.
"""
from __future__ import annotations

import random

import numpy as np
import torch


def set_seed(seed: int = 2025) -> None:
    """utils.py:6-16: seed python, numpy and torch (all devices)."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def compute_auc(y_true, y_pred) -> float:
    y = np.asarray(y_true, dtype=np.float64).ravel()
    s = np.asarray(y_pred, dtype=np.float64).ravel()
    if y.size != s.size:
        raise ValueError("y_true and y_pred differ in length")
    pos = y == 1
    n_pos = int(pos.sum())
    n_neg = y.size - n_pos
    if n_pos == 0 or n_neg == 0:
        return 0.5
    order = np.argsort(s, kind="mergesort")
    ss = s[order]
    # average rank of each tie group (1-based)
    starts = np.flatnonzero(np.r_[True, ss[1:] != ss[:-1]])
    ends = np.r_[starts[1:], ss.size]
    avg = (starts + ends + 1) / 2.0
    ranks_sorted = np.repeat(avg, ends - starts)
    ranks = np.empty_like(ranks_sorted)
    ranks[order] = ranks_sorted
    return float((ranks[pos].sum() - n_pos * (n_pos + 1) / 2.0) / (n_pos * n_neg))


def compute_logloss(y_true, y_pred, eps: float = 1e-15) -> float:
    """utils.py:29-32 (sklearn log_loss(labels=[0,1]) semantics, probabilities clipped to [eps, 1-eps])."""
    y = np.asarray(y_true, dtype=np.float64).ravel()
    p = np.clip(np.asarray(y_pred, dtype=np.float64).ravel(), eps, 1 - eps)
    return float(-np.mean(y * np.log(p) + (1 - y) * np.log(1 - p)))
