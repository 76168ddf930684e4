"""Inference / export: the counterpart of src/Prediction.py.

    python -m ctr_recommendation_amd.predict [--config ../config/fibinet_config.yaml]
        [--checkpoint ../checkpoints/FiBiNET_best.pth] [--out prediction_fibinet.csv]
        [--zip submission_fibinet.zip] [--batch-size 8192]

Same flow as the reference script (src/Prediction.py:55-126): the YAML config, ``build_model``,
a checkpoint whose ``module.`` prefixes (a DataParallel save) are stripped before a strict
``load_state_dict`` (:72-78), eval mode, batches of 8192 test rows through the inference
collator -- here :class:`~ctr_recommendation_amd.loader.DeviceLoader` in "inference" mode, whose
unknown-id rule is the reference's whole-batch zero fallback (:37-42) -- and the export: CSV
``ID,Task2`` plus a deflated zip of it (:115-126).  Checkpoints are read with
``torch.load(weights_only=True)``: tensors only, nothing executed from the file.
"""
from __future__ import annotations

import argparse
import os
import zipfile
from typing import Dict, Iterable

import numpy as np
import torch


def strip_module_prefix(state_dict: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """src/Prediction.py:77: ``{k.replace('module.', ''): v}`` (a DataParallel checkpoint)."""
    return {k.replace("module.", ""): v for k, v in state_dict.items()}


def load_checkpoint(path: str, map_location="cpu") -> Dict[str, torch.Tensor]:
    """The reference's checkpoint (App. B keys, optionally ``module.``-prefixed), tensors only."""
    sd = torch.load(path, map_location=map_location, weights_only=True)
    return strip_module_prefix(sd)


@torch.no_grad()
def predict(model, batches: Iterable[Dict[str, torch.Tensor]]) -> np.ndarray:
    """Probabilities of every batch, in order (src/Prediction.py:106-113).

    ``model``: the drop-in module (eval mode is set here) or a FiBiNETTrainer (its predict)."""
    if hasattr(model, "eval"):
        model.eval()
    fwd = model.predict if hasattr(model, "predict") and not isinstance(model, torch.nn.Module) else model
    preds = []
    for b in batches:
        preds.append(fwd(b).float().cpu().numpy())
    return np.concatenate(preds) if preds else np.zeros(0, dtype=np.float32)


def export_submission(predictions: np.ndarray, csv_path: str = "prediction_fibinet.csv",
                      zip_path: str = "submission_fibinet.zip") -> None:
    """CSV ``ID,Task2`` + zip (src/Prediction.py:115-126), written with the same pandas calls so
    the file is byte-identical to the reference's for the same predictions."""
    import pandas as pd
    sub = pd.DataFrame()
    sub["ID"] = range(len(predictions))
    sub["Task2"] = predictions
    sub.to_csv(csv_path, index=False)
    with zipfile.ZipFile(zip_path, "w", zipfile.ZIP_DEFLATED) as zf:
        zf.write(csv_path)


def _config_path(p):
    if p:
        return p
    for cand in ("../config/fibinet_config.yaml", "config/fibinet_config.yaml"):
        if os.path.exists(cand):
            return cand
    raise FileNotFoundError("no config: pass --config")


def main(argv=None) -> np.ndarray:
    import yaml
    from .loader import ColumnarDataset, DeviceLoader, ItemInfoTable
    from .model_fibinet import build_model

    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--config")
    ap.add_argument("--checkpoint")
    ap.add_argument("--out", default="prediction_fibinet.csv")
    ap.add_argument("--zip", default="submission_fibinet.zip")
    ap.add_argument("--batch-size", type=int, default=8192)          # src/Prediction.py:97
    args = ap.parse_args(argv)
    with open(_config_path(args.config)) as f:
        cfg = yaml.safe_load(f)
    dataset_cfg = cfg["dataset_config"][cfg["dataset_id"]]
    model_cfg = cfg[cfg["base_expid"]]
    device = torch.device("cuda")
    model = build_model(None, model_cfg)
    ckpt = args.checkpoint
    if ckpt is None:
        ckpt = "../checkpoints/FiBiNET_best.pth"
        if not os.path.exists(ckpt):
            ckpt = "checkpoints/FiBiNET_best.pth"
    model.load_state_dict(load_checkpoint(ckpt))                     # strict, like :78
    model.to(device).eval()
    info = ItemInfoTable.from_parquet(dataset_cfg["item_info"], device)
    test = ColumnarDataset.from_parquet(dataset_cfg["test_data"], device)
    loader = DeviceLoader(test, info, args.batch_size, shuffle=False, max_len=int(model_cfg.get("max_len", 20)),
                          mode="inference")
    preds = predict(model, loader)
    export_submission(preds, args.out, args.zip)
    print(f"wrote {args.out} and {args.zip} ({len(preds)} predictions)")
    return preds


if __name__ == "__main__":
    main()
