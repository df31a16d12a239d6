"""Lab (GPU, one device): the parts of a sharded rank's NF4 step (tools/shard_compute_probe.py) -- the shard's
dequantise alone, then each GEMM route (hgemm = dequantised weight reused + k_hgemm, library = torch.matmul on it,
fused = the one-kernel NF4 GEMM) at the chunk shapes (rows = 2048 and 4096) -- with k_hgemm's launch plan.
Usage: python tools/shard_parts_probe.py"""
import ctypes as ct
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import python_src_quants.functional as F  # noqa: E402

M, N, K = 4096, 4096, 11008
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
X = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)


def graph_us(fn, reps=5, iters=10):
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        fn()
    gr.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            gr.replay()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / iters)
    return statistics.median(ts)


def plan(m, n, k):
    out = (ct.c_int * 4)()
    F.lib.chgemm_tn_plan(ct.c_int(m), ct.c_int(n), ct.c_int(k), out)
    return tuple(out)


t0 = time.time()
while time.time() - t0 < 0.3:
    torch.matmul(X, X[:4096].t())
for world in (2, 4, 8):
    shard = N // world
    W = (torch.randn(shard, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    del W
    Wd = torch.empty(shard * K, device=dev, dtype=torch.bfloat16)
    tdq = graph_us(lambda: F._dequant_4bit_nested(q, st, Wd))
    line = f"shard {shard:4d}: dequantise {tdq:6.2f} us |"
    for rows in (2048, 4096):
        Y = torch.empty(rows, shard, device=dev, dtype=torch.bfloat16)
        F.gemm_4bit(X[:rows], q, st, out=Y, _route="hgemm")
        th = graph_us(lambda: F.gemm_4bit(X[:rows], q, st, out=Y, _route="hgemm", reuse_weight=True))
        F.gemm_4bit(X[:rows], q, st, out=Y, _route="library")
        tl = graph_us(lambda: F.gemm_4bit(X[:rows], q, st, out=Y, _route="library", reuse_weight=True))
        tf = graph_us(lambda: F.gemm_4bit(X[:rows], q, st, out=Y, _route="fused"))
        fl = 2.0 * rows * shard * K
        line += (f" rows {rows}: k_hgemm {th:6.2f} us ({fl / th / 1e6:5.0f} TF, plan {plan(rows, shard, K)}), "
                 f"library {tl:6.2f}, fused {tf:6.2f} |")
    print(line, flush=True)
