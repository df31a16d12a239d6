"""A/B of the 4-bit streaming dequantise's launch shape (cdequantize_set_stream_cfg: dwords per lane per pass, grid cap)
at the metric step's weight (4096 x 11008 NF4, nested statistics -> bf16), alone back to back and in the metric step's
order (dequantise, then k_hgemm at 4096 x 4096 x 11008), interleaved rounds after a clock ramp."""
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
ref = F.dequantize_4bit(q, st).view(-1)


def deq():
    F._dequant_4bit_nested(q, st, Wd)


def gemm():
    lib.chgemm_tn_bf16(ct.c_int32(M), ct.c_int32(N), ct.c_int32(K), F.get_ptr(X), ct.c_int32(K), F.get_ptr(Wd),
                       ct.c_int32(K), F.get_ptr(out), ct.c_int32(N))


cfgs = [(8, 0), (4, 0), (16, 0), (8, 1024), (8, 2048), (16, 1024), (4, 2048), (16, 512)]
for p, cap in cfgs:                       # correctness of every shape
    lib.cdequantize_set_stream_cfg(ct.c_int(p), ct.c_int(cap))
    Wd.zero_()
    deq()
    torch.cuda.synchronize()
    assert torch.equal(Wd, ref), (p, cap)
t_end = time.perf_counter() + 0.5
while time.perf_counter() < t_end:
    gemm()
    torch.cuda.synchronize()
best_alone = {c: 1e9 for c in cfgs}
best_step = {c: 1e9 for c in cfgs}
best_deq_in_step = {c: 1e9 for c in cfgs}
R = 20
for rnd in range(5):
    for c in cfgs:
        lib.cdequantize_set_stream_cfg(ct.c_int(c[0]), ct.c_int(c[1]))
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        deq()
        s.record()
        for _ in range(R):
            deq()
        e.record()
        e.synchronize()
        best_alone[c] = min(best_alone[c], s.elapsed_time(e) / R * 1e3)
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * R + 1)]
        evs[0].record()
        for i in range(R):
            deq()
            evs[2 * i + 1].record()
            gemm()
            evs[2 * i + 2].record()
        evs[-1].synchronize()
        best_step[c] = min(best_step[c], evs[0].elapsed_time(evs[-1]) / R * 1e3)
        d = sorted(evs[2 * i].elapsed_time(evs[2 * i + 1]) * 1e3 for i in range(R))
        best_deq_in_step[c] = min(best_deq_in_step[c], d[R // 2])
lib.cdequantize_set_stream_cfg(ct.c_int(8), ct.c_int(0))
print("p  cap   dequant alone  dequant in step (median)  step (dequant + k_hgemm)")
for c in cfgs:
    print(f"{c[0]:2d} {c[1]:5d}  {best_alone[c]:8.2f} us  {best_deq_in_step[c]:8.2f} us  {best_step[c]:8.2f} us")
