"""Lab (GPU): how much of the decode GEMV's time is its weight's trip from HBM -- gemv_4bit at 11008 x 4096 (nested NF4,
bf16) over 14 rotating weight copies (past the 256 MB MALL: HBM, as bench.py's decode leg) vs 1 copy replayed (its 23 MB
stays in the MALL) vs 14 copies where each call is preceded by a plain read of its weight (warmed, not timed apart).
HIP-graph replay, median of 5.  Usage: python tools/gemv_mall_probe.py"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import python_src_quants.functional as F  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(2)


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


for n, k in ((11008, 4096), (4096, 4096), (7168, 8192)):
    ws = []
    for _ in range(14):
        W = (torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
        del W
    x = torch.randn(1, k, device=dev, dtype=torch.bfloat16, generator=g)
    out = torch.empty(1, n, device=dev, dtype=torch.bfloat16)
    t14 = graph_us([lambda q=q, st=st: F.gemv_4bit(x, q.t(), out=out, state=st) for q, st in ws])
    q0, s0 = ws[0]
    t1 = graph_us([lambda: F.gemv_4bit(x, q0.t(), out=out, state=s0)] * 14)
    print(f"{n} x {k}: 14 rotating copies (HBM) {t14:6.2f} us   one copy replayed (MALL) {t1:6.2f} us", flush=True)
    del ws
