"""A/B (GPU): store policy of the metric step's two big writes -- the 4-bit streaming dequantise's bf16 weight
(cdequantize_set_store_policy: 0 default write-back, 1 non-temporal, 2 device-scope write-through) and k_hgemm's C
(chgemm_set_c_store: 0 write-back, 1 write-through) -- at the metric step's weight (4096 x 11008 NF4, nested
statistics): (a) the dequantise alone back to back, (b) the metric step itself (functional.gemm_4bit: dequantise, then
k_hgemm at 4096 x 4096 x 11008), (c) the int8 igemmlt + dequant at the same shape; HIP-graph replay, interleaved
rounds after a clock ramp; outputs checked equal."""
import ctypes as ct
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import python_src_quants.functional as F  # noqa: E402
from python_src_quants.cextension import lib  # noqa: E402

M, N, K = 4096, 4096, 11008
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
X = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
Wd = torch.empty(N * K, device=dev, dtype=torch.bfloat16)
out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
ref_w = F.dequantize_4bit(q, st).view(-1)
ref_y = F.gemm_4bit(X, q, st)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(reps):
            fn()
    gr.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        gr.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / (5 * reps)


A8 = (torch.randn(M, K, device=dev, generator=g) * 2).half()
Wt = (torch.randn(N, K, device=dev, generator=g) * 0.05).half()
CB, _, SCB, _, _ = F.double_quant(Wt)
CA, _, SCA, _, _ = F.double_quant(A8)
out8 = torch.empty(M, N, dtype=torch.float16, device=dev)
ref8 = F.igemmlt_dequant(CA, CB, SCA, SCB)
arms = [(0, 0), (1, 0), (2, 0), (0, 1), (2, 1)]          # (dequantise store, C store)
for dq, cw in arms:
    lib.cdequantize_set_store_policy(ct.c_int(dq))
    lib.chgemm_set_c_store(ct.c_int(cw))
    Wd.zero_()
    F._dequant_4bit_nested(q, st, Wd)
    y = F.gemm_4bit(X, q, st, out=out)
    F.igemmlt_dequant(CA, CB, SCA, SCB, out=out8)
    torch.cuda.synchronize()
    assert torch.equal(Wd, ref_w), (dq, cw)
    assert torch.equal(out, ref_y), (dq, cw)
    assert torch.equal(out8, ref8), (dq, cw)
t0 = time.time()
while time.time() - t0 < 0.5:
    F.gemm_4bit(X, q, st, out=out)
torch.cuda.synchronize()
res = {a: {"alone": [], "step": [], "int8": []} for a in arms}
for rnd in range(5):
    for a in arms:
        lib.cdequantize_set_store_policy(ct.c_int(a[0]))
        lib.chgemm_set_c_store(ct.c_int(a[1]))
        res[a]["alone"].append(timed(lambda: F._dequant_4bit_nested(q, st, Wd), 20))
        res[a]["step"].append(timed(lambda: F.gemm_4bit(X, q, st, out=out), 10))
        res[a]["int8"].append(timed(lambda: F.igemmlt_dequant(CA, CB, SCA, SCB, out=out8), 10))
lib.cdequantize_set_store_policy(ct.c_int(0))
lib.chgemm_set_c_store(ct.c_int(0))
names = {0: "write-back", 1: "non-temporal", 2: "write-through"}
for a in arms:
    al, s_, i8 = (sorted(res[a][k])[2] for k in ("alone", "step", "int8"))
    print(f"dequantise {names[a[0]]:13s} C {names[a[1] * 2]:13s}: dequantise alone {al:6.2f} us   metric step {s_:7.2f} us "
          f"({2 * M * N * K / s_ / 1e6:.1f} TFLOP/s)   int8 igemmlt+dequant {i8:7.2f} us", flush=True)
