"""A/B of the gather kernel with and without hot-row LDS staging (north star: "LDS staging of hot
rows", SURVEY 8(d)'s Zipf(1.05) ids), kernel time only: per batch the hot list is built untimed
(fbn_hot_rows), then fbn_fields_fwd_hot and fbn_fields_fwd are each timed with HIP events on the
same inputs (C3: B = 8192, d = 128, L = 20, V = 1.25 M, bf16 mode, 8 batches cycled).  Prints the
staged-row share of the history slots.  Usage: python tools/ab_hot_gather.py [zipf] [tau ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ctr_recommendation_amd import ops
from ctr_recommendation_amd._lib import call, ptr
from ctr_recommendation_amd.data import make_device_batches
from ctr_recommendation_amd.model_fibinet import build_model

dev = torch.device("cuda", 0)
B, d, L, V = 8192, 128, 20, 1_250_000
zipf = float(sys.argv[1]) if len(sys.argv) > 1 else 1.05
taus = [int(x) for x in sys.argv[2:]] or [2, 4, 8, 16]
p = {k: v.to(dev) for k, v in build_model(None, {"embedding_dim": d, "vocab_size": 4}).state_dict().items()}
p["item_emb.weight"] = torch.randn((V, d), device=dev)
batches = make_device_batches(8, B, V, L, dev, seed=3, zipf=zipf)
fc = ops.FwdConfig(d=d, L=L, training=True, p_drop=0.0, bf16=True, bilinear_each=False, R=3)
a = ops.forward(p, batches[0][0], fc, None, labels=batches[0][1], loss_denom=float(B))
st = ops._lib.stream_handle(dev)
cnt = torch.zeros(V, dtype=torch.int32, device=dev)
hot = torch.zeros(256, dtype=torch.int32, device=dev)
hot_n = torch.zeros(1, dtype=torch.int32, device=dev)
H = 8192 // d
E = p["item_emb.weight"]


def args(batch):
    return (ptr(batch["item_id"]), ptr(batch["item_seq"]), ptr(batch["likes_level"]), ptr(batch["views_level"]),
            ptr(a["hmm"]), ptr(p["mm_proj.1.weight"]), ptr(p["mm_proj.1.bias"]), ops.LN_EPS, ptr(p["cate_emb.weight"]),
            p["cate_emb.weight"].shape[0], ptr(E), V)


def tail():
    return (ptr(p["senet.excitation.0.weight"]), ptr(p["senet.excitation.0.bias"]), ptr(p["senet.excitation.2.weight"]),
            ptr(p["senet.excitation.2.bias"]), 3, ptr(a["X"]), None, ptr(a["Vc16"]), None, 15 * d, 1, ptr(a["a"]),
            ptr(a["cnt"]), ptr(a["err"]), None, None, B, L, d)


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(1_000_000)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3


for tau in taus:
    t_hot, t_plain, share, nh = [], [], [], []
    for rep in range(3):
        for batch, _ in batches:
            call("fbn_hot_rows", ptr(batch["item_id"]), ptr(batch["item_seq"]), B, L, V, ptr(cnt), ptr(hot), ptr(hot_n),
                 H, tau, 0, st)
            torch.cuda.synchronize()
            n = min(int(hot_n.item()), H)
            nh.append(n)
            seq = batch["item_seq"]
            share.append(float(torch.isin(seq[seq > 0], hot[:n]).float().mean()) if n else 0.0)
            t_hot.append(timed(lambda: call("fbn_fields_fwd_hot", *args(batch), *tail(), ptr(hot), ptr(hot_n), H, st)))
            t_plain.append(timed(lambda: call("fbn_fields_fwd", *args(batch), None, *tail(), 0, st)))
            call("fbn_hot_rows", ptr(batch["item_id"]), ptr(batch["item_seq"]), B, L, V, ptr(cnt), None, ptr(hot_n), H,
                 tau, 1, st)
    k = len(batches)
    th, tp = sorted(t_hot[k:])[len(t_hot[k:]) // 2], sorted(t_plain[k:])[len(t_plain[k:]) // 2]
    print(f"zipf {zipf} tau {tau}: staged rows {sum(nh) / len(nh):.0f}, staged share of history slots "
          f"{sum(share) / len(share):.3f} | gather with LDS staging {th:.1f} us, plain {tp:.1f} us")
