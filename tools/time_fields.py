"""Time fbn_fields_fwd and fbn_fields_bwd (with its partial reductions) at C3 shapes (B=8192,
d=128, L=20, V=1.25M, bf16), cycling 8 batches (their 88 MB of rows each do not stay in the
Infinity Cache between uses); FBN_FIELDS_HCH selects the gather's rows-in-flight chunk,
FBN_FIELDS_NOBUF=1 the global-load form, FBN_GATHER_HOT=<tau> the hot-row LDS staging; ZIPF=<s>
draws the ids from Zipf(s) (SURVEY 8(d)'s popularity skew)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ctr_recommendation_amd import ops
from ctr_recommendation_amd.data import make_device_batches
from ctr_recommendation_amd.model_fibinet import build_model

dev = torch.device("cuda", 0)
B, d, L, V = 8192, 128, 20, 1_250_000
cfg = {"embedding_dim": d, "vocab_size": 4}
small = build_model(None, cfg).state_dict()
p = {k: v.to(dev) for k, v in small.items()}
p["item_emb.weight"] = torch.randn((V, d), device=dev)
g = {k: torch.zeros_like(v) for k, v in p.items() if v.is_floating_point()}
ZIPF = float(os.environ.get("ZIPF", "0"))
batches = make_device_batches(8, B, V, L, dev, seed=3, zipf=ZIPF)
gvec = torch.zeros((B, 2, d), device=dev)
a = {}
fc = ops.FwdConfig(d=d, L=L, training=True, p_drop=0.0, bf16=True, bilinear_each=False, R=3)
probe = {}
for i in range(30):
    batch, labels = batches[i % len(batches)]
    torch.cuda._sleep(2_000_000)
    a = ops.forward(p, batch, fc, None, acts=a, probe=probe, labels=labels, loss_denom=float(B))
    ops.backward(p, batch, a, a["gout"], g, fc, gvec=gvec, probe=probe)
torch.cuda.synchronize()


def avg(name):
    ev = probe[name][10:]
    return sum(s.elapsed_time(e) for s, e in ev) / len(ev)


fwd, bwd = avg("fields_fwd"), avg("fields_bwd")
byts = ((L + 1) * d * 4 + (L + 3) * 8 + 4 * d * 4) * B
print(f"zipf={ZIPF} HCH={os.environ.get('FBN_FIELDS_HCH', 'default')} nobuf={os.environ.get('FBN_FIELDS_NOBUF', 0)} "
      f"hot={os.environ.get('FBN_GATHER_HOT', 0)}: fields_fwd {fwd * 1e3:.1f} us ({byts / fwd / 1e6 / 8000:.3f} "
      f"of 8 TB/s)  fields_bwd {bwd * 1e3:.1f} us")
