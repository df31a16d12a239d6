"""Lab (GPU): per-wave timeline of the few-token kernel (gemm4bit_fewtok.hip ABL 128 variant, 48-row workgroups, 8
waves) at 11008 x 4096 nested NF4, M tokens, mid-stream over 14 rotating weight copies.  Stamps (s_memrealtime, 10 ns)
relative to the earliest wave start: start, loads issued, table barrier, group 0 / 1 / 2 landed, compute done, end.
Usage: python tools/fewtok32_timeline.py [M] [ABL extra bits, e.g. 7]"""
import os
import sys
os.environ.setdefault("BNB_HIP_LIBRARY", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                   "bitsandbytes-sycl_amd", "build", "libbitsandbytes_hip_lab.so"))   # lab hooks: `make -C bitsandbytes-sycl_amd/csrc lab`

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bitsandbytes-sycl_amd"))
from python_src_quants import functional as F  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 8
extra = int(sys.argv[2]) if len(sys.argv) > 2 else 0
dev = torch.device("cuda", 0)
gen = torch.Generator(device=dev).manual_seed(3)
n_out, k_in = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (11008, 4096)
ws = []
for _ in range(14):
    W = (torch.randn(n_out, k_in, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
    ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
    del W
x = torch.randn(m, k_in, device=dev, dtype=torch.bfloat16, generator=gen)
out = torch.empty(m, n_out, device=dev, dtype=torch.bfloat16)
F.GEMM_4BIT_GEMV_TOKENS = 1
rows_per_wg = 48 if n_out > 16 * 256 else 16
nwg = (n_out + rows_per_wg - 1) // rows_per_wg
buf = torch.zeros(nwg * 8 * 8, dtype=torch.int64, device=dev)
F.set_fewtok_mode(16 + 128 + extra)
for it in range(3):
    for i, (q, st) in enumerate(ws):
        if it == 2 and i == 7:
            F.lib.cgemm_4bit_fewtok_timeline(F.get_ptr(buf))
        F.gemm_4bit(x, q, st, out=out)
        if it == 2 and i == 7:
            torch.cuda.synchronize()
            F.lib.cgemm_4bit_fewtok_timeline(None)
torch.cuda.synchronize()
F.set_fewtok_mode(0)
t = buf.view(nwg * 8, 8).cpu().numpy().astype(np.int64)
t = t[t[:, 0] > 0]
t0 = t[:, 0].min()
names = ["start", "issued", "table barrier", "group0 landed", "group1 landed", "group2 landed", "compute done", "end"]
print(f"M={m} ABL extra {extra}: {len(t)} waves; times in us after the first wave start (p5 / p50 / p95 / max)")
for i, nm in enumerate(names):
    v = t[:, i]
    v = v[v > 0]
    if len(v) == 0:
        continue
    v = (v - t0) / 100.0
    print(f"  {nm:14s} {np.percentile(v, 5):6.2f} {np.percentile(v, 50):6.2f} {np.percentile(v, 95):6.2f} {v.max():6.2f}")
tw = buf.view(nwg, 8, 8).cpu().numpy().astype(np.int64)
live = tw[:, :, 0].min(axis=1) > 0
st = tw[live, :, 0]
wg_start = (st.min(axis=1) - t0) / 100.0
intra = (st.max(axis=1) - st.min(axis=1)) / 100.0
print(f"  workgroup start (first wave) p5/p50/p95/max {np.percentile(wg_start, 5):.2f} {np.percentile(wg_start, 50):.2f} "
      f"{np.percentile(wg_start, 95):.2f} {wg_start.max():.2f}; spread of starts within a workgroup p50/max "
      f"{np.percentile(intra, 50):.2f} {intra.max():.2f}")
