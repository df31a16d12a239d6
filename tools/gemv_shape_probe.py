"""Per-shape decode GEMV time (gemv_4bit, nested NF4 bs 64, bf16), `copies` distinct weights replayed from one HIP
graph, GB/s over packed weights + statistics; per kernel choice (cgemv_4bit_set_kernel: 3 = balanced / dot, 21..24 = the
wide kernel with 1..4 chunks per lane), max |difference| to the first choice relative to its rms.
Usage: [GEMV_KNOBS=3,21,22,23,24] [GEMV_TWO_LDS=bytes] python tools/gemv_shape_probe.py [NxK ...]"""
import os
import sys
os.environ.setdefault("BNB_HIP_LIBRARY", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                   "bitsandbytes-sycl_amd", "build", "libbitsandbytes_hip_lab.so"))   # lab hooks: `make -C bitsandbytes-sycl_amd/csrc lab`

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bitsandbytes-sycl_amd"))
from python_src_quants import functional as F  # noqa: E402

SHAPES = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]] or [
    (11008, 4096), (1024, 8192), (128, 8192), (3584, 8192), (1024, 28672), (4096, 4096), (8192, 8192), (4096, 11008)]


KNOBS = [int(v) for v in os.environ.get("GEMV_KNOBS", "3,21,22,23,24").split(",")]


def graph_us(calls, iters=20):
    for c in calls:
        c()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for c in calls:
            c()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(5):
        s.record()
        for _ in range(iters):
            g.replay()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / iters / len(calls))
    return best


def main():
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(1)
    if os.environ.get("GEMV_TWO_LDS"):          # lab: LDS bytes up to which the balanced kernel runs 2 per CU
        F.lib.cgemv_4bit_set_two_per_cu_lds(int(os.environ["GEMV_TWO_LDS"]))
    for n, k in SHAPES:
        copies = max(2, min(64, int(400e6 // (n * k // 2))))
        ws = []
        for _ in range(copies):
            W = (torch.randn(n, k, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
            ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
            del W
        x = torch.randn(1, k, device=dev, dtype=torch.bfloat16, generator=gen)
        out = torch.empty(1, n, device=dev, dtype=torch.bfloat16)
        b = n * k // 2 + n * k // 64 + n * k // 64 // 256 * 4 + 1024
        line, ref = f"{n}x{k} ({copies} copies):", None
        for knob in KNOBS:
            F.lib.cgemv_4bit_set_kernel(knob)
            t = graph_us([(lambda q=q, st=st: F.gemv_4bit(x, q.t(), out=out, state=st)) for q, st in ws])
            y = F.gemv_4bit(x, ws[0][0].t(), state=ws[0][1]).float()
            ref = y if ref is None else ref
            d = (y - ref).abs().max().item() / ref.pow(2).mean().sqrt().item()
            line += f"  k{knob} {t:6.2f} us {b / t / 1e3:5.0f} GB/s (d {d:.0e})"
        F.lib.cgemv_4bit_set_kernel(0)
        print(line, flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
