"""Decode GEMV (M = 1) across layer shapes, per kernel choice (cgemv_4bit_set_kernel knob: 0 = default,
1 = the 4-waves-x-R-rows kernel only, others = A/B variants), GPU time per call from HIP-graph replay over enough
rotating weight copies to defeat the 256 MB MALL.  One graph per knob, replayed in alternation (ABAB...) so clock
and warm-up drift fall on every knob alike; median of the replays.
Usage: [GEMV_KNOBS=0,1] python tools/gemv_sweep.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "bitsandbytes-sycl_amd"))
import python_src_quants.functional as F  # noqa: E402

KNOBS = [int(v) for v in os.environ.get("GEMV_KNOBS", "0,1").split(",")]
if os.environ.get("GEMV_SHAPES"):
    SHAPES_ENV = [tuple(int(a) for a in s.split("x")) for s in os.environ["GEMV_SHAPES"].split(",")]
else:
    SHAPES_ENV = None
SHAPES = [(11008, 4096), (4096, 4096), (4096, 11008), (14336, 4096), (4096, 14336), (1024, 4096),
          (28672, 8192), (8192, 8192), (32000, 4096), (5000, 7680)]


def capture(fns):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for f in fns:
            f()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for f in fns:
                f()
    torch.cuda.synchronize()
    return g


def replay_us(g, n):
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


for nested in (False, True):
    for (n, k) in (SHAPES_ENV or SHAPES):
        bytes_per = n * k // 2 + (n * k // 64) * (1 if nested else 4)
        copies = max(2, min(64, (400 << 20) // bytes_per + 1))
        W = (torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16)
        ws = [F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=nested) for _ in range(copies)]
        del W
        x = torch.randn(1, k, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(1, n, device="cuda", dtype=torch.bfloat16)
        fns = [(lambda q=q, st=st: F.gemv_4bit(x, q.t(), out=out, state=st)) for (q, st) in ws]
        graphs = []
        for knob in KNOBS:
            F.lib.cgemv_4bit_set_kernel(knob)
            graphs.append(capture(fns))
        F.lib.cgemv_4bit_set_kernel(0)
        for g in graphs:
            replay_us(g, len(fns))
        ts = [[] for _ in KNOBS]
        for _ in range(15):
            for i, g in enumerate(graphs):
                ts[i].append(replay_us(g, len(fns)))
        res = [sorted(t)[len(t) // 2] for t in ts]
        print(f"{'nested' if nested else 'plain '} {n:6d} x {k:6d}  " + "  ".join(
            f"knob{kn} {t:6.2f} us ({bytes_per / t / 1e3:5.0f} GB/s)" for kn, t in zip(KNOBS, res)), flush=True)
        del ws, graphs
        torch.cuda.empty_cache()
