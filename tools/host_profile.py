"""Where the host time of one eager C3 (or EG_D/EG_V/EG_B) trainer step goes (cProfile over 40 steps with next_batch,
the bench's eager form).  Prints the median enqueue time per step and the top functions."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ctr_recommendation_amd.data import make_device_batches
from ctr_recommendation_amd.trainer import FiBiNETTrainer

dev = torch.device("cuda", 0)
# C3 by default; EG_D / EG_V / EG_B for another config (C2: 16 / 1000000 / 4096)
d, V, B = int(os.environ.get("EG_D", 128)), int(os.environ.get("EG_V", 1_250_000)), int(os.environ.get("EG_B", 8192))
cfg = {"embedding_dim": d, "vocab_size": V, "compute_dtype": "bf16"}
tr = FiBiNETTrainer(cfg, total_steps=400, batch_size=B, device=dev)
nb = 8
batches = make_device_batches(nb, B, V, 20, dev, seed=1)
for i in range(10):
    tr.step(*batches[i % nb], next_batch=batches[(i + 1) % nb][0])
torch.cuda.synchronize()
host = []
for i in range(20):
    torch.cuda._sleep(5_000_000)      # the GPU stays behind: pure host enqueue time
    t0 = time.perf_counter()
    tr.step(*batches[i % nb], next_batch=batches[(i + 1) % nb][0])
    host.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
print(f"median host enqueue {sorted(host)[len(host) // 2] * 1e3:.3f} ms per step")
if os.environ.get("HP_NOPROF") == "1":
    sys.exit(0)
pr = cProfile.Profile()
pr.enable()
for i in range(40):
    tr.step(*batches[i % nb], next_batch=batches[(i + 1) % nb][0])
    if i % 8 == 7:
        torch.cuda.synchronize()
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
st.sort_stats("cumulative").print_stats(25)
