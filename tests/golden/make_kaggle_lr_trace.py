"""Extract the OneCycleLR trace (and per-epoch AUC log) that the reference's Kaggle run printed.

Source (read as text, not executed): /root/reference/Notebooks/train_predict_kaggle.ipynb, the
output of `python train_fibinet.py` (lines "Epoch e | Step s | Loss: l | LR: lr", printed by
src/train_fibinet.py:127-129 every 200 steps, and "Epoch e | Train Loss | Valid AUC").
Writes tests/golden/kaggle_lr_trace.json (data only).
"""
import json
import os
import re

NB = "/root/reference/Notebooks/train_predict_kaggle.ipynb"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kaggle_lr_trace.json")

nb = json.load(open(NB))
text = "".join("".join(o.get("text", [])) for c in nb["cells"] for o in c.get("outputs", []))
steps = [dict(epoch=int(e), step=int(s), loss=float(l), lr=float(lr))
         for e, s, l, lr in re.findall(r"Epoch (\d+) \| Step (\d+) \| Loss: ([0-9.]+) \| LR: ([0-9.]+)", text)]
aucs = [dict(epoch=int(e), train_loss=float(l), valid_auc=float(a))
        for e, l, a in re.findall(r"Epoch (\d+) \| Train Loss: ([0-9.]+) \| Valid AUC: ([0-9.]+)", text)]
json.dump({"source": "Notebooks/train_predict_kaggle.ipynb (Kaggle T4 run of src/train_fibinet.py)",
           "config": {"learning_rate": 1e-3, "epochs": 40, "batch_size": 4096},
           "lr_trace": steps, "epoch_log": aucs}, open(OUT, "w"), indent=1)
print(len(steps), "lr points,", len(aucs), "epochs ->", OUT)
