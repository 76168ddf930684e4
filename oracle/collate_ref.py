"""CPU restatement of the reference data path -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates, with the same pandas / numpy / torch calls the reference makes:

* ParquetDataset.load_data ......... src/dataloader.py:21-48 (object columns -> 2-D arrays, one
                                     np.column_stack: a common dtype, float64 with the label)
* BatchCollator.__call__ ........... src/dataloader.py:54-121 (default_collate, column split,
                                     .loc lookup of item_emb_d128, last-max_len item_seq, label pop)
* InferenceCollator.__call__ ....... src/Prediction.py:21-52 (reindex().fillna(0); any exception ->
                                     the whole batch's mm vectors are zeros)
* the export ....................... src/Prediction.py:115-126 (CSV ID,Task2 + zip)

The reference files themselves are never imported or run; these functions are
checked against hand-built expectations in tests/test_loader.py.
"""
from __future__ import annotations

import zipfile
from typing import Dict, List, Tuple

import numpy as np
import pandas as pd
import torch
from torch.utils.data.dataloader import default_collate


def load_data(data_path: str) -> Tuple[np.ndarray, Dict]:
    """ParquetDataset.load_data (src/dataloader.py:21-48): (darray, column_index)."""
    df = pd.read_parquet(data_path)
    column_index, arrays, idx = {}, [], 0
    for col in df.columns:
        if df[col].dtype == "object":
            array = np.array(df[col].to_list())
            if len(array.shape) == 1:
                array = array.reshape(-1, 1)
            seq_len = array.shape[1]
            column_index[col] = [i + idx for i in range(seq_len)]
            idx += seq_len
        else:
            array = df[col].to_numpy().reshape(-1, 1)
            column_index[col] = idx
            idx += 1
        arrays.append(array)
    return np.column_stack(arrays), column_index


def _split(batch_rows: List[np.ndarray], column_index: Dict) -> Dict[str, torch.Tensor]:
    batch_tensor = default_collate(batch_rows)                       # src/dataloader.py:71
    out = {}
    for col, idx in column_index.items():                            # :76-80
        out[col] = batch_tensor[:, idx] if isinstance(idx, list) else batch_tensor[:, idx].squeeze(-1)
    return out


class BatchCollatorRef:
    """BatchCollator (src/dataloader.py:53-121)."""

    def __init__(self, max_len: int, column_index: Dict, item_info_path: str):
        self.max_len, self.column_index = max_len, column_index
        self.item_info = pd.read_parquet(item_info_path).set_index("item_id")     # :59

    def __call__(self, batch_rows):
        batch_dict = _split(batch_rows, self.column_index)
        item_ids = batch_dict["item_id"].numpy()                      # :84
        batch_item_info = self.item_info.loc[item_ids]                # :91 (KeyError on unknown ids)
        emb_vals = np.stack(batch_item_info["item_emb_d128"].values)  # :94
        batch_dict["item_emb_d128"] = torch.tensor(emb_vals, dtype=torch.float32)
        if "item_seq" in batch_dict:                                  # :111-116
            seq = batch_dict["item_seq"]
            if seq.shape[1] > self.max_len:
                seq = seq[:, -self.max_len:]
            batch_dict["item_seq"] = seq.long()
        labels = batch_dict.pop("label").float()                      # :119
        return batch_dict, labels


class InferenceCollatorRef:
    """InferenceCollator (src/Prediction.py:21-52)."""

    def __init__(self, max_len: int, column_index: Dict, item_info_path: str):
        self.max_len, self.column_index = max_len, column_index
        self.item_info = pd.read_parquet(item_info_path).set_index("item_id")

    def __call__(self, batch_rows):
        batch_dict = _split(batch_rows, self.column_index)
        item_ids = batch_dict["item_id"].numpy()
        try:                                                          # :37-42
            batch_item_info = self.item_info.reindex(item_ids).fillna(0)
            emb_vals = np.stack(batch_item_info["item_emb_d128"].values)
        except Exception:
            emb_vals = np.zeros((len(item_ids), 128))
        batch_dict["item_emb_d128"] = torch.tensor(emb_vals, dtype=torch.float32)
        if "item_seq" in batch_dict:
            seq = batch_dict["item_seq"]
            if seq.shape[1] > self.max_len:
                seq = seq[:, -self.max_len:]
            batch_dict["item_seq"] = seq.long()
        return batch_dict


def batches(darray: np.ndarray, collator, batch_size: int):
    """DataLoader(shuffle=False) over ParquetDataset rows (src/dataloader.py:14-19, :139-143)."""
    for lo in range(0, darray.shape[0], batch_size):
        yield collator([darray[i, :] for i in range(lo, min(lo + batch_size, darray.shape[0]))])


def export_submission(predictions: np.ndarray, csv_path: str, zip_path: str) -> None:
    """src/Prediction.py:115-126."""
    sub = pd.DataFrame()
    sub["ID"] = range(len(predictions))
    sub["Task2"] = predictions
    sub.to_csv(csv_path, index=False)
    with zipfile.ZipFile(zip_path, "w", zipfile.ZIP_DEFLATED) as zf:
        zf.write(csv_path)
