"""Lab (GPU, one device): the per-rank compute of bench.py's sharded NF4 step at world = 1, 2, 4, 8 -- this rank's
[N / world, K] shard, the tokens in `chunks` row chunks (the first call dequantises the shard, the later ones reuse it),
no collective -- against the ideal 1 / world of the world-1 step.  HIP-graph replay, median of 5 after a clock ramp.
Prints the route gemm_4bit takes per shape.  Usage: python tools/shard_compute_probe.py"""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import python_src_quants.functional as F  # noqa: E402
import bench  # noqa: E402

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


base = None
for world in (1, 2, 4, 8):
    shard = N // world
    W = (torch.randn(shard, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    del W
    chunks = 2 if world > 1 else 1
    Mc = M // chunks
    Y = torch.empty(M, shard, device=dev, dtype=torch.bfloat16)

    def step():
        for c in range(chunks):
            F.gemm_4bit(X[c * Mc:(c + 1) * Mc], q, st, out=Y[c * Mc:(c + 1) * Mc], reuse_weight=c > 0)
    t0 = time.time()
    while time.time() - t0 < 0.3:
        step()
    torch.cuda.synchronize()
    t = graph_us(step)
    if base is None:
        base = t
    route = bench.gemm_kernel_name(Mc, shard)
    print(f"world {world}: shard {shard:4d} x {K}, {chunks} chunk(s) of {Mc} rows: {t:7.2f} us per rank "
          f"(ideal {base / world:6.2f}, efficiency {base / world / t:.2f})  route: {route}", flush=True)
