"""MicroLens-shaped synthetic batches for tests and the benchmark.

The batch_dict contract is the reference collator's (src/dataloader.py:69-121):
``item_id`` [B] int64, ``item_seq`` [B, max_len] int64 (the LAST max_len items, left-padded
with 0), ``likes_level`` / ``views_level`` [B] int64 in [0, 10], ``user_id`` [B] int64
(unused by the model), ``item_emb_d128`` [B, 128] float32; labels [B] float32.

Generation (seeded, numpy ``default_rng``):
* item_id ~ U[1, V); history: n_valid ~ U{0..L}, left-padded, valid slots ~ U[1, V);
* likes/views ~ U{0..10}; user_id ~ U[1, 20000);
* item_emb_d128: N(0,1) rows L2-normalised (mimics Notebooks/task-1.ipynb:237-239);
* label ~ Bernoulli(sigmoid(score)), score a fixed hash of (item_id mod 97, likes, views) plus
  a term in the mm vector, so that AUC is non-trivial.
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np
import torch


def make_batch_np(rng: np.random.Generator, B: int, V: int, L: int = 20, n_cate: int = 11,
                  zipf: float = 0.0, signal: str = "hash") -> Tuple[Dict[str, np.ndarray], np.ndarray]:
    """signal "hash": the planted score of SURVEY §8(d); "fields": a score a few training steps
    can learn (the cate levels and the mm vector carry it) -- for AUC-parity tests, where an
    AUC near 0.5 would say nothing."""
    if zipf > 0:
        item = (rng.zipf(1.0 + zipf, size=B) % (V - 1)) + 1
    else:
        item = rng.integers(1, V, size=B)
    n_valid = rng.integers(0, L + 1, size=B)
    hist = rng.integers(1, V, size=(B, L))
    slot = np.arange(L)[None, :]
    seq = np.where(slot >= (L - n_valid)[:, None], hist, 0)        # left-padded
    likes = rng.integers(0, n_cate, size=B)
    views = rng.integers(0, n_cate, size=B)
    user = rng.integers(1, 20000, size=B)
    mm = rng.standard_normal((B, 128)).astype(np.float32)
    mm /= np.linalg.norm(mm, axis=1, keepdims=True)
    if signal == "fields":
        score = (likes - 5) / 1.5 - (views - 5) / 2.5 + 12.0 * mm[:, 0]
    else:
        score = (((item % 97) * 7 + likes * 3 - views * 2) % 11 - 5) / 2.5 + 2.0 * mm[:, 0]
    label = (rng.random(B) < 1.0 / (1.0 + np.exp(-score))).astype(np.float32)
    batch = {
        "item_id": item.astype(np.int64),
        "item_seq": seq.astype(np.int64),
        "likes_level": likes.astype(np.int64),
        "views_level": views.astype(np.int64),
        "user_id": user.astype(np.int64),
        "item_emb_d128": mm,
    }
    return batch, label


def to_torch(batch: Dict[str, np.ndarray], label: np.ndarray, device="cpu"):
    return {k: torch.from_numpy(np.ascontiguousarray(v)).to(device) for k, v in batch.items()}, \
        torch.from_numpy(label).to(device)


def make_batch(seed: int, B: int, V: int, L: int = 20, device="cpu", zipf: float = 0.0, signal: str = "hash"):
    rng = np.random.default_rng(seed)
    b, y = make_batch_np(rng, B, V, L, zipf=zipf, signal=signal)
    return to_torch(b, y, device)


def make_device_batches(n: int, B: int, V: int, L: int, device, seed: int = 2025, zipf: float = 0.0):
    """Pre-generate ``n`` batches directly on the device (benchmark input, HBM-resident).

    zipf = s > 0: item and history ids follow Zipf(s) over the V - 1 ids (SURVEY §8(d)'s
    Zipf(1.05) popularity skew): rank k has probability k^-s / H, ranks mapped to ids by a fixed
    random permutation (hot rows scattered over the table); else ids ~ U[1, V)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    draw = None
    if zipf > 0:
        ranks = torch.arange(1, V, device=device, dtype=torch.float64)
        cdf = torch.cumsum(ranks.pow(-zipf), 0)
        cdf = (cdf / cdf[-1]).float()
        perm = torch.randperm(V - 1, generator=g, device=device) + 1

        def draw(shape):
            u = torch.rand(shape, generator=g, device=device)
            k = torch.searchsorted(cdf, u.reshape(-1)).clamp_(max=V - 2)
            return perm[k].reshape(shape).to(torch.int64)
    out = []
    for _ in range(n):
        if draw is not None:
            item = draw((B,))
            hist = draw((B, L))
        else:
            item = torch.randint(1, V, (B,), generator=g, device=device, dtype=torch.int64)
            hist = None
        n_valid = torch.randint(0, L + 1, (B,), generator=g, device=device)
        if hist is None:
            hist = torch.randint(1, V, (B, L), generator=g, device=device, dtype=torch.int64)
        slot = torch.arange(L, device=device)[None, :]
        seq = torch.where(slot >= (L - n_valid)[:, None], hist, torch.zeros_like(hist))
        likes = torch.randint(0, 11, (B,), generator=g, device=device, dtype=torch.int64)
        views = torch.randint(0, 11, (B,), generator=g, device=device, dtype=torch.int64)
        mm = torch.randn((B, 128), generator=g, device=device)
        mm = mm / mm.norm(dim=1, keepdim=True)
        score = (((item % 97) * 7 + likes * 3 - views * 2) % 11 - 5).float() / 2.5 + 2.0 * mm[:, 0]
        label = (torch.rand((B,), generator=g, device=device) < torch.sigmoid(score)).float()
        out.append(({"item_id": item, "item_seq": seq, "likes_level": likes, "views_level": views,
                     "item_emb_d128": mm.contiguous()}, label))
    return out


def write_microlens_parquet(out_dir: str, n_train: int, n_valid: int = 0, n_test: int = 0, n_items: int = 5000,
                            seq_width: int = 20, seed: int = 2025, item_id_stride: int = 1,
                            missing_ids=(), signal: str = "fields") -> Dict[str, str]:
    """Synthetic MicroLens_1M_x1-shaped parquet files (the schema of config/fibinet_config.yaml:30-37):
    train / valid / test with columns user_id, item_seq (list of seq_width ids, left-padded with 0),
    likes_level, views_level, item_id, label (test: no label), and item_info.parquet with item_id
    and item_emb_d128 (list of 128 float32, L2-normalised).  Item ids are 1 + k * item_id_stride
    (non-contiguous when the stride is > 1); ids in ``missing_ids`` are left out of item_info.
    Returns the dataset_config-style paths."""
    import os

    import pyarrow as pa
    import pyarrow.parquet as pq

    os.makedirs(out_dir, exist_ok=True)
    rng = np.random.default_rng(seed)
    ids = 1 + np.arange(n_items, dtype=np.int64) * item_id_stride
    emb = rng.standard_normal((n_items, 128)).astype(np.float32)
    emb /= np.linalg.norm(emb, axis=1, keepdims=True)
    keep = ~np.isin(ids, np.asarray(list(missing_ids), dtype=np.int64))
    info = pa.table({"item_id": pa.array(ids[keep]),
                     "item_emb_d128": pa.array(list(emb[keep]), type=pa.list_(pa.float32()))})
    paths = {"item_info": os.path.join(out_dir, "item_info.parquet")}
    pq.write_table(info, paths["item_info"])
    for split, n in (("train", n_train), ("valid", n_valid), ("test", n_test)):
        if n <= 0:
            continue
        k = rng.integers(0, n_items, size=n)
        item = ids[k]
        n_valid = rng.integers(0, seq_width + 1, size=n)
        hist = ids[rng.integers(0, n_items, size=(n, seq_width))]
        slot = np.arange(seq_width)[None, :]
        seq = np.where(slot >= (seq_width - n_valid)[:, None], hist, 0)
        likes = rng.integers(0, 11, size=n)
        views = rng.integers(0, 11, size=n)
        mm0 = emb[k, 0]
        score = (likes - 5) / 1.5 - (views - 5) / 2.5 + 12.0 * mm0 if signal == "fields" else \
            (((item % 97) * 7 + likes * 3 - views * 2) % 11 - 5) / 2.5 + 2.0 * mm0
        label = (rng.random(n) < 1.0 / (1.0 + np.exp(-score))).astype(np.float32)
        cols = {"user_id": pa.array(rng.integers(1, 20000, size=n)),
                "item_seq": pa.array(list(seq.astype(np.int64)), type=pa.list_(pa.int64())),
                "likes_level": pa.array(likes.astype(np.int64)),
                "views_level": pa.array(views.astype(np.int64)),
                "item_id": pa.array(item)}
        if split != "test":
            cols["label"] = pa.array(label)
        path = os.path.join(out_dir, f"{split}.parquet")
        pq.write_table(pa.table(cols), path)
        paths[f"{split}_data"] = path
    return paths
