"""The bf16 dgrad GEMMs with the weight read K-contiguous (the transposed image the step builds
today) or k-major (the weight's own layout, ds_read_b64_tr_b16 fragments), interleaved rounds:
  dc  = dh1 Wa   (8192 x 1920 x 512, bf16 out)
  dh1 = dh2 Wb   (8192 x 512 x 256, f32 out)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ctr_recommendation_amd import ops
from ctr_recommendation_amd._lib import call, ptr

dev = "cuda"
bf = torch.bfloat16
B, KC, H1, H2 = 8192, 1920, 512, 256
dh1 = torch.randn((B, H1), device=dev).to(bf)
Wa = torch.randn((H1, KC), device=dev).to(bf)
WaT = Wa.T.contiguous()
dc = torch.empty((B, KC), device=dev, dtype=bf)
dh2 = torch.randn((B, H2), device=dev).to(bf)
Wb = torch.randn((H2, H1), device=dev).to(bf)
WbT = Wb.T.contiguous()
out = torch.empty((B, H1), device=dev)
st = ops._lib.stream_handle()
arms = {
    "dc  WaT (K-contig)": lambda: call("fbn_gemm_bf16out", ptr(dh1), ptr(WaT), ptr(dc), B, KC, H1, H1, H1, KC, 0, 1, st),
    "dc  Wa  (k-major) ": lambda: call("fbn_gemm_bf16out", ptr(dh1), ptr(Wa), ptr(dc), B, KC, H1, H1, KC, KC, 0, 0, st),
    "dh1 WbT (K-contig)": lambda: ops.gemm(dh2, WbT, out, B, H1, H2, H2, H2, H1, False, True, stream=st),
    "dh1 Wb  (k-major) ": lambda: ops.gemm(dh2, Wb, out, B, H1, H2, H2, H1, H1, False, False, stream=st),
}
res = {k: [] for k in arms}
for _ in range(5):
    for name, fn in arms.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(1_000_000)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name].append(e0.elapsed_time(e1) / 20 * 1e3)
for name, v in res.items():
    v = sorted(v)
    print(f"{name}: median {v[len(v) // 2]:6.2f} us  min {v[0]:6.2f} us")
call("fbn_gemm_bf16out", ptr(dh1), ptr(WaT), ptr(dc), B, KC, H1, H1, H1, KC, 0, 1, st)
r1 = dc.clone()
call("fbn_gemm_bf16out", ptr(dh1), ptr(Wa), ptr(dc), B, KC, H1, H1, KC, KC, 0, 0, st)
ops.gemm(dh2, WbT, out, B, H1, H2, H2, H2, H1, False, True, stream=st)
o1 = out.clone()
ops.gemm(dh2, Wb, out, B, H1, H2, H2, H1, H1, False, False, stream=st)
torch.cuda.synchronize()
print("dc identical:", torch.equal(r1, dc), " dh1 identical:", torch.equal(o1, out))
