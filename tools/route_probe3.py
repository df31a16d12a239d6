"""Static-route probe (GPU): for each prefill shape, the time of every route of functional.gemm_4bit forced with
_route= ("hgemm" = dequantise + k_hgemm, "library" = dequantise + torch.matmul, "library_tn" = dequantise + rocBLAS
with the per-shape solution search, "fused" = the one-kernel NF4 GEMM, split-K on small grids), nested NF4 bs 64,
bf16, medians of 5 interleaved rounds of 10 calls; prints the static rule's pick beside the fastest.
Usage: python tools/route_probe3.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402

SHAPES = [  # (rows, out features, in features)
    (4096, 1024, 8192), (4096, 128, 8192), (4096, 3584, 8192), (4096, 1024, 28672),    # 70B 8-way shards
    (2048, 1024, 8192), (2048, 3584, 8192), (2048, 1024, 28672),
    (4096, 2048, 8192), (4096, 2048, 28672), (4096, 7168, 8192),                         # 70B 4-way shards
    (2048, 4096, 4096), (2048, 11008, 4096), (2048, 4096, 11008),                         # 7B at 2048 tokens
    (4096, 4096, 11008), (4096, 11008, 4096), (1024, 4096, 11008), (512, 11008, 4096), (256, 11008, 4096), (128, 11008, 4096), (96, 11008, 4096),
    (200, 8192, 2048),
]


def timed(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    for M, N, K in SHAPES:
        W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
        del W
        X = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        routes = ["hgemm", "library", "library_tn", "fused"]
        res = {r: [] for r in routes}
        for r in routes:                       # warm (code objects, rocBLAS search, workspaces)
            F.gemm_4bit(X, q, st, out=out, _route=r)
        torch.cuda.synchronize()
        for _ in range(5):
            for r in routes:
                res[r].append(timed(lambda r=r: F.gemm_4bit(X, q, st, out=out, _route=r)))
        med = {r: sorted(v)[2] for r, v in res.items()}
        best = min(med, key=med.get)
        static = F.gemm_4bit_static_route(M, N, K)
        line = f"{M:6d}x{N:6d}x{K:6d} static {static:10s} best {best:10s} " + " ".join(
            f"{r} {med[r]:8.1f}" for r in routes)
        print(line, flush=True)
        del q, st, X, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
