"""Where the metric step's time goes beyond its two kernels (lab, GPU).

Times the bench's metric step (functional.gemm_4bit at M=4096, N=4096, K=11008, nested NF4 -> HIP dequantise +
hipBLASLt GEMM) four ways, interleaved over several rounds so clock drift hits every arm alike:
  plain   : K back-to-back calls, wall clock (no events)
  events  : the same with the bench's per-stage events (events=) and a step-level event pair
  sparse  : per-stage events on every 10th call only
  chain   : one event per step boundary (K + 1 in all) + per-stage events on every 10th call (bench.py's form)
  graph   : the step captured once in a HIP graph and replayed
Usage: python tools/step_overhead.py [steps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bitsandbytes-sycl_amd"))
from python_src_quants import functional as F  # noqa: E402

M, N, K, BS = 4096, 4096, 11008, 64


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=BS, quant_type="nf4", compress_statistics=True)
    del W
    Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

    def run_plain(n):
        for _ in range(n):
            F.gemm_4bit(X, q, st, out=Y)

    kev = []

    def run_events(n, every=1):
        for i in range(n):
            if i % every == 0:
                s = torch.cuda.Event(enable_timing=True)
                e = torch.cuda.Event(enable_timing=True)
                s.record()
                ev = []
                F.gemm_4bit(X, q, st, out=Y, events=ev)
                e.record()
                kev.append(ev)
            else:
                F.gemm_4bit(X, q, st, out=Y)

    # warm + clock ramp
    t_end = time.perf_counter() + 1.0
    while time.perf_counter() < t_end:
        run_plain(10)
        torch.cuda.synchronize()

    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        F.gemm_4bit(X, q, st, out=Y)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            F.gemm_4bit(X, q, st, out=Y)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()

    def run_graph(n):
        for _ in range(n):
            g.replay()

    def run_chain(n):
        b = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
        b[0].record()
        for i in range(n):
            ev = [] if i % 10 == 0 else None
            F.gemm_4bit(X, q, st, out=Y, events=ev)
            b[i + 1].record()
            if ev is not None:
                kev.append(ev)

    arms = {"plain": run_plain, "events": run_events, "sparse": lambda n: run_events(n, 10), "chain": run_chain,
            "graph": run_graph}
    res = {k: [] for k in arms}
    for rnd in range(5):
        for name, fn in arms.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn(steps)
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / steps * 1e6)
    flops = 2.0 * M * N * K
    for name, v in res.items():
        v.sort()
        print(f"{name:7s} us/step: median {v[len(v) // 2]:.1f}  min {v[0]:.1f}  max {v[-1]:.1f}  "
              f"-> {flops / (v[len(v) // 2] * 1e-6) / 1e12:.0f} TFLOP/s")
    d = [sum(s.elapsed_time(e) for nm, s, e in ev if nm == "dequantize") * 1e3 for ev in kev]
    gm = [sum(s.elapsed_time(e) for nm, s, e in ev if nm == "gemm") * 1e3 for ev in kev]
    print(f"stage events: dequantize {sum(d) / len(d):.1f} us, gemm {sum(gm) / len(gm):.1f} us")


if __name__ == "__main__":
    main()
