"""In-process A/B of the eager C3 step over Python-level switches (module globals of trainer /
ops), alternating blocks of K steps per arm for R rounds on one trainer at steady state; prints
the median ms/step per arm (AB_ZIPF=s: Zipf(s) ids).  Usage: python tools/ab_step.py ARM [ARM ...] with ARM =
name:module.GLOBAL=value[;module.GLOBAL=value...] ('base' = no change; module env = an
environment variable the library reads per call), e.g.
  python tools/ab_step.py base claim_main:trainer._CLAIM_ON_SIDE=False"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ctr_recommendation_amd import ops, trainer as trmod
from ctr_recommendation_amd.data import make_device_batches
from ctr_recommendation_amd.trainer import FiBiNETTrainer

class _Env:
    """env.NAME=value arms: the C library reads some A/B knobs per call (getenv)."""
    def __getattr__(self, k):
        return os.environ.get(k)

    def __setattr__(self, k, v):
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = str(v)


mods = {"trainer": trmod, "ops": ops, "env": _Env()}
arms = []
for a in sys.argv[1:] or ["base"]:
    name, _, spec = a.partition(":")
    sets = []
    for kv in filter(None, spec.split(";")):
        k, v = kv.split("=")
        m, g = k.split(".")
        sets.append((mods[m], g, eval(v)))
    arms.append((name, sets))
dev = torch.device("cuda", 0)
V, B, K, R = 1_250_000, 8192, int(os.environ.get("AB_K", 40)), int(os.environ.get("AB_R", 6))
tr = FiBiNETTrainer({"embedding_dim": 128, "vocab_size": V, "compute_dtype": "bf16"}, total_steps=300 + 2 * R * K * len(arms),
                    batch_size=B, device=dev)
nb = 160
batches = make_device_batches(nb, B, V, 20, dev, seed=2025, zipf=float(os.environ.get("AB_ZIPF", "0")))
i = 0
for _ in range(280):
    tr.step(*batches[i % nb], next_batch=batches[(i + 1) % nb][0])
    i += 1
torch.cuda.synchronize()
base = {(m, g): getattr(m, g) for _, sets in arms for m, g, _ in sets}
res = {name: [] for name, _ in arms}
for rnd in range(R):
    for name, sets in arms:
        for (m, g), v in base.items():
            setattr(m, g, v)
        for m, g, v in sets:
            setattr(m, g, v)
        for _ in range(4):                      # settle
            tr.step(*batches[i % nb], next_batch=batches[(i + 1) % nb][0])
            i += 1
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            tr.step(*batches[i % nb], next_batch=batches[(i + 1) % nb][0])
            i += 1
        torch.cuda.synchronize()
        res[name].append((time.perf_counter() - t0) / K * 1e3)
for name, v in res.items():
    v = sorted(v)
    print(f"{name:16s} median {v[len(v) // 2]:.4f} ms/step  min {v[0]:.4f}  all {' '.join(f'{x:.4f}' for x in v)}")
