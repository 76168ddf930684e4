"""Time fbn_fields_fwd and fbn_fields_bwd (with its partial reductions) at C3 shapes (B=8192,
d=128, L=20, V=1.25M, bf16), cycling 8 batches (their 88 MB of rows each do not stay in the
Infinity Cache between uses); kernel spans from the library's kernel probes.

Arms (interleaved in one process, ROUNDS rounds; each arm sets environment knobs the library reads
per call), e.g.
    python tools/time_fields.py "plain:" "cmp10:FBN_FIELDS_CMP=1,FBN_FIELDS_HCH=10"
Knobs: FBN_FIELDS_HCH the history rows in flight per chunk, FBN_FIELDS_CMP=1 live slots compacted
first, FBN_FIELDS_NOBUF=1 global loads instead of the buffer resource, FBN_GATHER_HOT=<tau> hot-row LDS staging; env ZIPF=<s> draws Zipf(s) ids, D / B the shape."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ctr_recommendation_amd import ops
from ctr_recommendation_amd.data import make_device_batches
from ctr_recommendation_amd.model_fibinet import build_model

dev = torch.device("cuda", 0)
d = int(os.environ.get("D", "128"))
B = int(os.environ.get("B", "8192"))
L, V = 20, int(os.environ.get("V", "1250000"))
ROUNDS = int(os.environ.get("ROUNDS", "4"))
cfg = {"embedding_dim": d, "vocab_size": 4}
small = build_model(None, cfg).state_dict()
p = {k: v.to(dev) for k, v in small.items()}
p["item_emb.weight"] = torch.randn((V, d), device=dev)
g = {k: torch.zeros_like(v) for k, v in p.items() if v.is_floating_point()}
ZIPF = float(os.environ.get("ZIPF", "0"))
batches = make_device_batches(8, B, V, L, dev, seed=3, zipf=ZIPF)
gvec = torch.zeros((B, 2, d), device=dev)
fc = ops.FwdConfig(d=d, L=L, training=True, p_drop=0.0, bf16=True, bilinear_each=False, R=3)
arms = [a.split(":", 1) for a in (sys.argv[1:] or ["default:"])]
knobs = sorted({kv.split("=")[0] for _, spec in arms for kv in spec.split(",") if kv})
res = {name: {"fwd": [], "bwd": []} for name, _ in arms}
a = {}
for rnd in range(ROUNDS):
    for name, spec in arms:
        for k in knobs:
            os.environ.pop(k, None)
        for kv in (x for x in spec.split(",") if x):
            k, v = kv.split("=")
            os.environ[k] = v
        probe = {}
        for i in range(20):
            batch, labels = batches[i % len(batches)]
            torch.cuda._sleep(1_000_000)
            a = ops.forward(p, batch, fc, None, acts=a, probe=probe, labels=labels, loss_denom=float(B))
            ops.backward(p, batch, a, a["gout"], g, fc, gvec=gvec, probe=probe)
        torch.cuda.synchronize()
        for key, pn in (("fwd", "fields_fwd"), ("bwd", "fields_bwd")):
            ev = probe[pn][5:]
            res[name][key].append(sum(s.elapsed_time(e) for s, e in ev) / len(ev))
for k in knobs:
    os.environ.pop(k, None)
byts = ((L + 1) * d * 4 + (L + 3) * 8 + 4 * d * 4) * B
for name, spec in arms:
    f = sorted(res[name]["fwd"])
    bw = sorted(res[name]["bwd"])
    fm = f[len(f) // 2]
    print(f"d={d} B={B} zipf={ZIPF} {name} [{spec}]: fields_fwd median {fm * 1e3:.2f} us (rounds "
          f"{', '.join(f'{x * 1e3:.2f}' for x in res[name]['fwd'])}; {byts / fm / 1e6 / 8000:.3f} of 8 TB/s on "
          f"SURVEY 8(d)'s count)  fields_bwd {bw[len(bw) // 2] * 1e3:.2f} us", flush=True)
