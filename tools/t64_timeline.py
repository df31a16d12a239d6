"""Lab (GPU): per-wave timeline of the 33..64-token kernel (gemm4bit_t64.hip ABL 512 variant, 4 waves) at 11008 x 4096
nested NF4, M tokens, mid-stream over 14 rotating weight copies.  Stamps (s_memrealtime, 10 ns) relative to the earliest
wave start: start, prologue issued, table built, first half-group landed, loop done, DMA drained, outputs issued, outputs
landed.  Usage: python tools/t64_timeline.py [M]"""
import ctypes as ct
import os
import sys
os.environ.setdefault("BNB_HIP_LIBRARY", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                   "bitsandbytes-sycl_amd", "build", "libbitsandbytes_hip_lab.so"))   # lab hooks: `make -C bitsandbytes-sycl_amd/csrc lab`

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bitsandbytes-sycl_amd"))
from python_src_quants import functional as F  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda", 0)
gen = torch.Generator(device=dev).manual_seed(3)
n_out, k_in = 11008, 4096
ws = []
for _ in range(14):
    W = (torch.randn(n_out, k_in, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
    ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
    del W
x = torch.randn(m, k_in, device=dev, dtype=torch.bfloat16, generator=gen)
out = torch.empty(m, n_out, device=dev, dtype=torch.bfloat16)
nwg = 256
buf = torch.zeros(nwg * 4 * 8, dtype=torch.int64, device=dev)
prev = F.lib.cgemm_4bit_set_t64_mode(ct.c_int(16 + 512))
for it in range(3):
    for i, (q, st) in enumerate(ws):
        if it == 2 and i == 7:
            F.lib.cgemm_4bit_t64_timeline(F.get_ptr(buf))
        F.gemm_4bit(x, q, st, out=out)
        if it == 2 and i == 7:
            torch.cuda.synchronize()
            F.lib.cgemm_4bit_t64_timeline(None)
torch.cuda.synchronize()
F.lib.cgemm_4bit_set_t64_mode(ct.c_int(prev))
t = buf.view(nwg * 4, 8).cpu().numpy().astype(np.int64)
t = t[t[:, 0] > 0]
t0 = t[:, 0].min()
names = ["start", "prologue issued", "table built", "first landed", "loop done", "DMA drained", "outputs issued",
         "outputs landed"]
print(f"t64 M={m}: {len(t)} waves; us after the first wave start (p5 / p50 / p95 / max)")
for i, nm in enumerate(names):
    v = t[:, i]
    v = v[v > 0]
    if len(v) == 0:
        continue
    v = (v - t0) / 100.0
    print(f"  {nm:16s} {np.percentile(v, 5):6.2f} {np.percentile(v, 50):6.2f} {np.percentile(v, 95):6.2f} {v.max():6.2f}")
