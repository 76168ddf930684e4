"""Debug helper: per-parameter gradient error of the drop-in HIP module vs the CPU oracle."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ctr_recommendation_amd.data import make_batch
from ctr_recommendation_amd.model_fibinet import build_model
from oracle.fibinet_oracle import build_model as oracle_build

for d in (16, 128):
    cfg = {"embedding_dim": d, "vocab_size": 5000, "honour_config": True, "net_dropout": 0.0}
    torch.manual_seed(0); ref = oracle_build(None, cfg, honour_config=True)
    torch.manual_seed(0); hip = build_model(None, cfg).cuda().train()
    ref.train()
    batch, labels = make_batch(3, 128, 5000)
    lf = torch.nn.BCELoss()
    lf(ref(batch), labels).backward()
    lf(hip({k: v.cuda() for k, v in batch.items()}), labels.cuda()).backward()
    rg = {n: p.grad for n, p in ref.named_parameters()}
    for n, p in hip.named_parameters():
        if rg[n] is None:
            print(d, n, "ref None; hip", None if p.grad is None else "set"); continue
        g = p.grad.cpu()
        sc = rg[n].abs().max().item()
        print(f"d={d} {n:30s} scale={sc:.3e} err={(g-rg[n]).abs().max().item():.3e}")
