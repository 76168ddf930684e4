"""GPU-bound time of an eager C3 (or EG_D/EG_V/EG_B) step: the host enqueues 20 steps while the GPU is held by a
sleep kernel, so the steps then run back to back whatever the host's enqueue rate; compared
with the same 20 steps enqueued live (host and GPU racing) and with their host enqueue time."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ctr_recommendation_amd.data import make_device_batches
from ctr_recommendation_amd.trainer import FiBiNETTrainer

dev = torch.device("cuda", 0)
# C3 by default; EG_D / EG_V / EG_B for another config (C2: 16 / 1000000 / 4096)
d, V, B, K = (int(os.environ.get("EG_D", 128)), int(os.environ.get("EG_V", 1_250_000)),
              int(os.environ.get("EG_B", 8192)), 20)
tr = FiBiNETTrainer({"embedding_dim": d, "vocab_size": V, "compute_dtype": "bf16"}, total_steps=2000,
                    batch_size=B, device=dev)
nb = 160
batches = make_device_batches(nb, B, V, 20, dev, seed=2025)
i = 0
for _ in range(280):                       # steady state of the lazy table Adam (2F steps)
    tr.step(*batches[i % nb], next_batch=batches[(i + 1) % nb][0])
    i += 1
torch.cuda.synchronize()
for rnd in range(3):
    # live: host and GPU race
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for _ in range(K):
        tr.step(*batches[i % nb], next_batch=batches[(i + 1) % nb][0])
        i += 1
    th = time.perf_counter() - t0
    e1.record()
    torch.cuda.synchronize()
    live = e0.elapsed_time(e1) / K
    # queued: the GPU held by a sleep until all K steps are enqueued
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(60_000_000)
    e0.record()
    for _ in range(K):
        tr.step(*batches[i % nb], next_batch=batches[(i + 1) % nb][0])
        i += 1
    e1.record()
    torch.cuda.synchronize()
    q = e0.elapsed_time(e1) / K
    print(f"round {rnd}: live {live:.4f} ms/step (host enqueue {th / K * 1e3:.4f}), GPU-bound (pre-queued) {q:.4f} ms/step")
