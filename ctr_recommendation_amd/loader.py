"""HBM-resident data path: ParquetDataset + BatchCollator + MMCTRDataLoader
(src/dataloader.py:10-142) and InferenceCollator (src/Prediction.py:21-52), MI355X-first.

The reference reads a parquet split into ONE numpy array (np.column_stack coerces every column
to a common dtype, float64 once the float label is in: src/dataloader.py:21-48), then per batch,
in 4 worker processes: default_collate of the rows, a pandas ``.loc`` of ``item_emb_d128`` by
``item_id`` (:91-95), the last-``max_len`` truncation of ``item_seq`` (:111-116), and pageable H2D
copies in the train loop (src/train_fibinet.py:109-111) -- about 1e6 samples/s at best.

Here the split is read once, column by column (pyarrow), and moved to HBM (MicroLens-1M train:
3.6 M rows, ~0.7 GB of 288 GB); the item_info table (``item_id`` -> 128 floats) sits in HBM behind
a dense id -> row index.  A batch is ONE ``fbn_collate`` launch that gathers every column by the
epoch permutation and the item_info row of every item id (HIP, ``csrc/collate.hip``); batches come
out on the device already, in the reference's batch_dict contract (``item_id``, ``item_seq``,
``likes_level``, ``views_level``, ``user_id`` int64; ``item_emb_d128`` float32; labels float32).

Errors follow the reference: an item id without an item_info row raises ``KeyError`` in training
(the ``.loc`` of src/dataloader.py:104-106; raised by :meth:`DeviceLoader.check`, lazily, from a
device flag), while inference zeroes the whole batch's mm vectors (src/Prediction.py:37-42: the
``reindex().fillna(0)`` + ``np.stack`` except branch).  Ragged list columns raise ``ValueError``
(``np.array`` of ragged lists does).
"""
from __future__ import annotations

import math
from typing import Dict, Iterator, Optional, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr

INT_COLS = ("item_id", "likes_level", "views_level", "user_id")


def _list_column(col, name: str) -> np.ndarray:
    """A parquet list column as a 2-D array (equal-length lists only, as np.array(col_list))."""
    import pyarrow as pa
    arr = col.combine_chunks() if hasattr(col, "combine_chunks") else col
    if isinstance(arr, pa.ChunkedArray):
        arr = pa.concat_arrays(arr.chunks)
    offsets = np.asarray(arr.offsets)
    lens = np.diff(offsets)
    if len(lens) and (lens != lens[0]).any():
        raise ValueError(f"column {name!r}: lists of unequal length ({lens.min()}..{lens.max()}); "
                         "the reference's np.array(col_list) cannot stack them either")
    width = int(lens[0]) if len(lens) else 0
    vals = np.asarray(arr.flatten())
    return vals.reshape(len(lens), width)


def read_parquet_columns(path: str) -> Dict[str, np.ndarray]:
    """{column: array} of a parquet file; list columns become [rows, width] (src/dataloader.py:21-48)."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    t = pq.read_table(path)
    out = {}
    for name in t.column_names:
        col = t.column(name)
        if pa.types.is_list(col.type) or pa.types.is_large_list(col.type) or pa.types.is_fixed_size_list(col.type):
            out[name] = _list_column(col, name)
        else:
            out[name] = col.to_numpy()
    return out


class ItemInfoTable:
    """item_info (``item_id`` -> ``item_emb_d128``) in HBM behind a dense id -> row index
    (BatchCollator.__init__, src/dataloader.py:54-65: ``read_parquet(...).set_index("item_id")``),
    or, when the ids are sparse (largest id > DENSE_FACTOR x rows + 2^20), behind the sorted ids."""

    DENSE_FACTOR = 8
    DENSE_SLACK = 1 << 20

    def __init__(self, item_ids: np.ndarray, emb: np.ndarray, device):
        item_ids = np.asarray(item_ids, dtype=np.int64)
        emb = np.array(emb, dtype=np.float32, order="C")            # own, writable copy
        if emb.ndim != 2 or emb.shape[0] != item_ids.shape[0] or emb.shape[1] % 4:
            raise ValueError(f"item_info: {item_ids.shape[0]} ids vs embedding block {emb.shape}")
        if len(item_ids) and item_ids.min() < 0:
            raise ValueError("item_info: negative item_id")
        if len(np.unique(item_ids)) != len(item_ids):
            # .loc on a duplicated index returns several rows per id: the reference's np.stack then
            # no longer lines up with the batch
            raise ValueError("item_info: duplicate item_id")
        n_ids = int(item_ids.max()) + 1 if len(item_ids) else 0
        self.device = torch.device(device)
        self.dim = emb.shape[1]
        if n_ids <= self.DENSE_FACTOR * len(item_ids) + self.DENSE_SLACK:
            # dense id -> row index (MicroLens: ids 1..91 718, 0.4 MB)
            slot = np.full(max(1, n_ids), -1, dtype=np.int32)
            slot[item_ids] = np.arange(len(item_ids), dtype=np.int32)
            self.n_ids = n_ids
            self.sorted_ids = None
        else:
            # sparse / hashed ids: a dense index would be sized by the largest id -- the ids sorted
            # instead, and the collator binary-searches them
            order = np.argsort(item_ids, kind="stable")
            slot = order.astype(np.int32)
            self.n_ids = len(item_ids)
            self.sorted_ids = torch.from_numpy(np.ascontiguousarray(item_ids[order])).to(self.device)
        self.slot_of_id = torch.from_numpy(slot).to(self.device)
        self.emb = torch.from_numpy(emb).to(self.device)

    @classmethod
    def from_parquet(cls, path: str, device, column: str = "item_emb_d128") -> "ItemInfoTable":
        cols = read_parquet_columns(path)
        return cls(cols["item_id"], cols[column], device)


class ColumnarDataset:
    """A parquet split held column-wise in HBM (the role of ParquetDataset, src/dataloader.py:10-48).

    ``item_seq`` keeps its stored width Ls; collation keeps its last ``max_len`` columns."""

    def __init__(self, cols: Dict[str, np.ndarray], device, label_col: str = "label"):
        self.device = torch.device(device)
        n = len(cols["item_id"])
        self.n = n
        self.cols: Dict[str, torch.Tensor] = {}
        for name in INT_COLS:
            if name in cols:
                a = np.asarray(cols[name])
                if a.ndim != 1 or len(a) != n:
                    raise ValueError(f"column {name!r}: expected {n} scalars, got shape {a.shape}")
                self.cols[name] = torch.from_numpy(np.array(a, dtype=np.int64, order="C")).to(self.device)
        if "item_seq" in cols:
            s = np.asarray(cols["item_seq"])
            if s.ndim == 1:
                s = s.reshape(-1, 1)
            self.cols["item_seq"] = torch.from_numpy(np.array(s, dtype=np.int64, order="C")).to(self.device)
        self.has_label = label_col in cols
        if self.has_label:
            self.cols["label"] = torch.from_numpy(np.array(cols[label_col], dtype=np.float32, order="C")).to(
                self.device)

    @classmethod
    def from_parquet(cls, path: str, device, label_col: str = "label") -> "ColumnarDataset":
        if not path.endswith(".parquet") and not path.endswith(".pq"):
            path += ".parquet"                       # MMCTRDataLoader appends it (src/dataloader.py:130-131)
        return cls(read_parquet_columns(path), device, label_col)

    def __len__(self) -> int:
        return self.n


class DeviceLoader:
    """Batches of a :class:`ColumnarDataset` assembled in HBM (MMCTRDataLoader, src/dataloader.py:126-142).

    mode "train": yields (batch_dict, labels) like BatchCollator; mode "inference": yields batch_dict
    like InferenceCollator (labels dropped).  shuffle: a fresh device permutation per epoch (seeded;
    torch's DataLoader sampler stream cannot be matched and the reference does not fix it).
    rank / world: this rank's contiguous slice of every global batch (the multi-GPU trainer).
    """

    def __init__(self, dataset: ColumnarDataset, item_info: Optional[ItemInfoTable], batch_size: int,
                 shuffle: bool = False, max_len: int = 20, mode: str = "train", seed: int = 2025,
                 drop_last: bool = False, rank: int = 0, world: int = 1):
        if mode not in ("train", "inference"):
            raise ValueError(f"mode must be 'train' or 'inference', not {mode!r}")
        if mode == "train" and not dataset.has_label:
            raise ValueError("train mode needs a label column")
        if batch_size % world:
            raise ValueError(f"global batch {batch_size} does not split over {world} ranks")
        self.ds, self.info = dataset, item_info
        self.batch_size, self.shuffle, self.max_len, self.mode = batch_size, shuffle, max_len, mode
        self.drop_last, self.rank, self.world = drop_last, rank, world
        self.device = dataset.device
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        self.missing = torch.zeros(1, dtype=torch.int32, device=self.device)   # train: sticky KeyError flag
        self.epoch = 0

    def __len__(self) -> int:
        n = len(self.ds)
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def _perm(self) -> torch.Tensor:
        n = len(self.ds)
        if self.shuffle:
            return torch.randperm(n, generator=self.gen, device=self.device)
        return torch.arange(n, device=self.device)

    def collate(self, rows: torch.Tensor, flag: Optional[torch.Tensor] = None):
        """The batch of dataset rows `rows` (int64 device tensor): one fbn_collate launch."""
        _lib.require_hip(rows, "row index")
        B = rows.shape[0]
        dev = self.device
        c = self.ds.cols
        out = {"item_id": torch.empty(B, dtype=torch.int64, device=dev)}
        seq = c.get("item_seq")
        Ls = seq.shape[1] if seq is not None else 0
        L = min(Ls, self.max_len)
        if seq is not None:
            out["item_seq"] = torch.empty((B, L), dtype=torch.int64, device=dev)
        for k in ("likes_level", "views_level", "user_id"):
            if k in c:
                out[k] = torch.empty(B, dtype=torch.int64, device=dev)
        lab = torch.empty(B, dtype=torch.float32, device=dev) if (self.mode == "train") else None
        info = self.info
        if info is not None:
            out["item_emb_d128"] = torch.empty((B, info.dim), dtype=torch.float32, device=dev)
        flag = flag if flag is not None else self.missing
        call("fbn_collate", ptr(rows), B, ptr(c["item_id"]), ptr(seq), Ls, L, ptr(c.get("likes_level")),
             ptr(c.get("views_level")), ptr(c.get("user_id")), ptr(c["label"]) if lab is not None else None,
             ptr(info.slot_of_id) if info else None, info.n_ids if info else 0,
             ptr(info.sorted_ids) if info else None, ptr(info.emb) if info else None,
             info.dim if info else 0, ptr(out["item_id"]), ptr(out.get("item_seq")), ptr(out.get("likes_level")),
             ptr(out.get("views_level")), ptr(out.get("user_id")), ptr(lab), ptr(out.get("item_emb_d128")),
             ptr(flag), _lib.stream_handle(dev))
        return out, lab

    def __iter__(self) -> Iterator:
        perm = self._perm()
        self.epoch += 1
        n = len(self.ds)
        B = self.batch_size
        for i in range(len(self)):
            lo, hi = i * B, min(n, (i + 1) * B)
            # this rank's contiguous share of the global batch (the last, short batch splits too)
            share = -(-(hi - lo) // self.world)
            rlo, rhi = lo + self.rank * share, min(hi, lo + (self.rank + 1) * share)
            rows = perm[rlo:rhi]
            if self.mode == "inference":
                flag = torch.zeros(1, dtype=torch.int32, device=self.device)
                out, _ = self.collate(rows, flag)
                if "item_emb_d128" in out:
                    # src/Prediction.py:39-42: one unknown id zeroes the whole batch's mm vectors
                    call("fbn_collate_zero_if", ptr(out["item_emb_d128"]), out["item_emb_d128"].numel(), ptr(flag),
                         _lib.stream_handle(self.device))
                yield out
            else:
                yield self.collate(rows)

    def check(self, group=None, world: int = 1) -> None:
        """Raise the KeyError the reference's collator would have raised (one 4-byte read).

        world > 1: collective -- the flag is MAX-all-reduced first, so every rank raises at the same
        step (a rank that raised alone would leave the others blocked in the next step's
        collectives until the communicator's timeout)."""
        flag = self.missing
        if world > 1:
            import torch.distributed as dist
            flag = self.missing.clone()
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        if int(flag.item()):
            raise KeyError("item_id(s) of a batch are not in item_info (src/dataloader.py:104-106)")


def make_loaders(dataset_cfg: Dict, model_cfg: Dict, device, rank: int = 0, world: int = 1,
                 seed: int = 2025) -> Tuple[DeviceLoader, DeviceLoader, ItemInfoTable]:
    """train / valid loaders from the reference config surface (src/train_fibinet.py:40-61)."""
    bs = int(model_cfg.get("batch_size", 4096))
    max_len = int(model_cfg.get("max_len", 20))
    info = ItemInfoTable.from_parquet(dataset_cfg["item_info"], device)
    tr = DeviceLoader(ColumnarDataset.from_parquet(dataset_cfg["train_data"], device), info, bs, shuffle=True,
                      max_len=max_len, seed=seed, rank=rank, world=world)
    va = DeviceLoader(ColumnarDataset.from_parquet(dataset_cfg["valid_data"], device), info, bs, shuffle=False,
                      max_len=max_len, seed=seed, rank=rank, world=world)
    return tr, va, info
