"""Stand-alone timings of the sharded step's owner-side kernels (fbn_sumsq_sparse, fbn_owner_fold,
fbn_owner_gather) on synthetic one-rank fixed-capacity data: HIP events over R launches each.
  python tools/time_owner.py [n_slots]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ctr_recommendation_amd import _lib
from ctr_recommendation_amd._lib import call, ptr

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 14657
D, V = 128, 1250000
R = 50
g = torch.Generator(device="cpu").manual_seed(0)
ids = torch.randint(1, V, (n,), generator=g, dtype=torch.int32)
ids[torch.rand(n, generator=g) < 0.15] = -1                      # empty slots
ids = ids.to(dev)
mp = torch.full((V,), -1, dtype=torch.int32, device=dev)
slot_row = torch.full((n,), -1, dtype=torch.int32, device=dev)
call("fbn_owner_claim", ptr(ids), n, ptr(mp), ptr(slot_row), 0, _lib.stream_handle())
wire = torch.randn((n, D), device=dev).bfloat16()
ring = torch.zeros((2, n, D), device=dev)
step = torch.zeros(1, dtype=torch.int32, device=dev)
cell = torch.zeros(2, dtype=torch.int64, device=dev)
extra = torch.zeros((n, D), device=dev)
out = torch.zeros(64, dtype=torch.float64, device=dev)
part = torch.zeros(8192, dtype=torch.float64, device=dev)
E = torch.randn((V, D), device=dev)
reply = torch.empty((n, D), device=dev).bfloat16()
st = _lib.stream_handle()


flush = torch.empty(1 << 28, device=dev)        # 1 GiB: evicts L2 and the MALL between cold launches


def timeit(name, fn):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(R):
        fn()
    b.record()
    torch.cuda.synchronize()
    hot = a.elapsed_time(b) / R * 1e3
    cold = 0.0
    for _ in range(10):
        flush.fill_(1.0)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        cold += a.elapsed_time(b) * 1e3 / 10
    print(f"{name:28s} hot {hot:8.1f} us   cold {cold:8.1f} us", flush=True)


timeit("owner_fold", lambda: call("fbn_owner_fold", ptr(ids), n, 0, ptr(mp), ptr(slot_row), ptr(wire), 1, None, 0, 0,
                                  ptr(ring), 2, n * D, ptr(step), ptr(cell), ptr(extra), D, ptr(part), None, st))
timeit("sumsq_flagged", lambda: call("fbn_sumsq_flagged", ptr(slot_row), n, ptr(cell), ptr(extra), D, ptr(part),
                                     ptr(out), None, 0, st))
timeit("sumsq_sparse (cell)", lambda: call("fbn_sumsq_sparse", ptr(cell), ptr(extra), ptr(slot_row), 1 | 0x20000, n, D,
                                           ptr(out), None, 0, st))
timeit("sumsq_sparse (direct)", lambda: call("fbn_sumsq_sparse", ptr(ring), ptr(extra), ptr(slot_row), 1, n, D,
                                             ptr(out), None, 0, st))
timeit("owner_gather", lambda: call("fbn_owner_gather", ptr(ids), n, ptr(E), ptr(reply), None, None, 0, D, 1, st))
