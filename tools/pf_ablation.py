"""What bounds the next-batch prefetch (adam_prefetch2_kernel, C3, uniform ids, steady state):
its launch timed alone (serialised probe steps: side work on the main stream behind a GPU sleep)
as is, without its arithmetic (FBN_PF_ABL=1: rows loaded and stored unchanged) and without its
row traffic (FBN_PF_ABL=2: the replay on zero rows, nothing stored), and with groups of 8 rows
(3; 4 = that without row traffic).  The ablations leave the
table wrong: only their launch times mean anything.  Prints the median launch time per arm."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ctr_recommendation_amd.data import make_device_batches
from ctr_recommendation_amd.trainer import FiBiNETTrainer

dev = torch.device("cuda", 0)
V, B = 1_250_000, 8192
tr = FiBiNETTrainer({"embedding_dim": 128, "vocab_size": V, "compute_dtype": "bf16"}, total_steps=2000,
                    batch_size=B, device=dev)
nb = 160
batches = make_device_batches(nb, B, V, 20, dev, seed=2025)
i = 0
for _ in range(280):
    tr.step(*batches[i % nb], next_batch=batches[(i + 1) % nb][0])
    i += 1
torch.cuda.synchronize()
side = tr.side
tr.side = torch.cuda.current_stream(dev)
res = {}
for rnd in range(3):
    for arm in ("real", "1", "2", "3", "4"):
        if arm == "real":
            os.environ.pop("FBN_PF_ABL", None)
        else:
            os.environ["FBN_PF_ABL"] = arm
        probe = {}
        for _ in range(6):
            torch.cuda._sleep(20_000_000)
            tr.step(*batches[i % nb], next_batch=batches[(i + 1) % nb][0], probe=probe)
            i += 1
        torch.cuda.synchronize()
        ts = [a.elapsed_time(e) * 1e3 for a, e in probe.get("adam_prefetch", [])]
        res.setdefault(arm, []).extend(ts)
os.environ.pop("FBN_PF_ABL", None)
tr.side = side
names = {"real": "prefetch as is", "1": "no arithmetic (rows in / out)", "2": "no row traffic (arithmetic)",
         "3": "groups of 8 rows", "4": "groups of 8, no row traffic"}
for arm, v in res.items():
    v = sorted(v)
    print(f"{names[arm]:32s} median {v[len(v) // 2]:.1f} us  min {v[0]:.1f}  n {len(v)}")
