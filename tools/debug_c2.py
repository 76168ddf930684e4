"""Bisect a drop-in gradient deviation at a config shape (debug aid): train-mode forward
intermediates vs the oracle, run-to-run determinism of the HIP gradients.

  python tools/debug_c2.py d V B
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ctr_recommendation_amd import ops
from ctr_recommendation_amd.data import make_batch
from ctr_recommendation_amd.model_fibinet import build_model
from oracle.fibinet_oracle import build_model as oracle_build

d, V, B = (int(x) for x in sys.argv[1:4])
dev = torch.device("cuda:0")
cfg = {"embedding_dim": d, "vocab_size": V, "honour_config": True, "net_dropout": 0.0}
torch.manual_seed(0)
ref = oracle_build(None, cfg, honour_config=True).train()
torch.manual_seed(0)
hip = build_model(None, cfg).to(dev).train()
b, y = make_batch(11, B, V)
db = {k: v.to(dev) for k, v in b.items()}
# oracle intermediates
with torch.no_grad():
    x = ref.fields(b)
    v = ref.senet(x)
    pairs = ref.bilinear(v)
    c = torch.cat([v.reshape(B, -1), pairs.reshape(B, -1)], 1)
    h1pre = ref.mlp[0](c)
p = {k: t.contiguous() for k, t in hip.state_dict().items()}
cfgf = ops.FwdConfig(d=d, L=20, training=True, p_drop=0.0)
a = ops.forward(p, db, cfgf, None)
torch.cuda.synchronize()


def cmp(name, h, r):
    h = h.cpu().float()
    print(f"{name}: max|d| {(h - r).abs().max().item():.3e}  max|r| {r.abs().max().item():.3e}  "
          f"argmax row {int((h - r).abs().reshape(h.shape[0], -1).max(1).values.argmax())}")


cmp("X[:,3] item", a["X"][:, 0], x[:, 3])
cmp("X[:,5] hist", a["X"][:, 1], x[:, 5])
cmp("c (compact V1..V5)", a["c"][:, :5 * d], c[:, d:6 * d])
cmp("c pairs", a["c"][:, 5 * d:], torch.cat([c[:, 6 * d + 5 * d:]], 1))
cmp("h1pre", a["h1pre"], h1pre)
lh = ref(b, return_logits=True).detach()
cmp("logits", a["logits"], lh)
# determinism of the drop-in gradients
gs = []
for rep in range(2):
    hip.zero_grad()
    torch.nn.BCELoss()(hip(db), y.to(dev)).backward()
    gs.append({n: q.grad.detach().clone() for n, q in hip.named_parameters() if q.grad is not None})
for n in gs[0]:
    dd = (gs[0][n] - gs[1][n]).abs().max().item()
    if dd > 0:
        print("nondeterministic", n, dd)
print("done")
