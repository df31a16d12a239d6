"""Lab (GPU): per-launch decode time of the Llama-2-70B rank-shard shapes (the four launches of bench.py's
decode_fused leg: q/k/v 1280 x 8192, o 1024 x 8192, gate/up 7168 x 8192, down 1024 x 28672), nested NF4 bs 64, one
token, over 8 rotating weight copies per shape (HIP-graph replay, median of 5), through gemv_4bit, plus the few-token
kernel forced (set_fewtok_mode(2)) on the same call where it applies.
Usage: python tools/decode70_probe.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bitsandbytes-sycl_amd"))
from python_src_quants import functional as F  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(5)
SHAPES = [tuple(int(v) for v in t.split('x')) for t in os.environ.get('DP_SHAPES', '1280x8192,1024x8192,7168x8192,1024x28672').split(',')]
COPIES = 8


def graph_us(calls, reps=5, iters=10):
    for c in calls:
        c()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for c in calls:
            c()
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
        ts.append(s.elapsed_time(e) * 1e3 / iters / len(calls))
    return statistics.median(ts)


for n, k in SHAPES:
    ws = []
    for _ in range(COPIES):
        W = (torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
        del W
    x = torch.randn(1, k, device=dev, dtype=torch.bfloat16, generator=g)
    out = torch.empty(1, n, device=dev, dtype=torch.bfloat16)
    wbytes = n * k // 2 + n * k // 64 + n * k // 64 // 256 * 4
    line = f"{n:5d} x {k:5d} ({wbytes / 1e6:5.1f} MB):"
    F.set_fewtok_mode(1)
    t = graph_us([lambda q=q, st=st: F.gemv_4bit(x, q.t(), out=out, state=st) for q, st in ws])
    line += f"  gemv_4bit {t:6.2f} us ({wbytes / t / 1e3:5.0f} GB/s)"
    if os.environ.get("DP_WIDE"):
        F.lib.cgemv_4bit_set_kernel(2)
        tw = graph_us([lambda q=q, st=st: F.gemv_4bit(x, q.t(), out=out, state=st) for q, st in ws])
        F.lib.cgemv_4bit_set_kernel(0)
        line += f"  wide(forced) {tw:6.2f} us"
    if not os.environ.get("DP_WIDE"):
        F.set_fewtok_mode(2)
        t2 = graph_us([lambda q=q, st=st: F.gemm_4bit(x, q, st, out=out) for q, st in ws])
        line += f"  fewtok(forced) {t2:6.2f} us"
    F.set_fewtok_mode(0)
    print(line, flush=True)
    del ws
