"""Route sweep (GPU) for the static rule of functional.gemm_4bit: rows x (out features, in features) over the prefill
routes "hgemm" (dequantise + k_hgemm, split-K on small grids), "fused" (one-kernel NF4 GEMM) and "library_tn"
(dequantise + rocBLAS, for reference), nested NF4 bs 64, bf16; medians of 3 interleaved rounds of 5 calls (us).
Usage: python tools/route_sweep4.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402

WEIGHTS = [(4096, 4096), (11008, 4096), (4096, 11008), (1024, 8192), (3584, 8192), (1024, 28672), (512, 11008),
           (128, 8192), (8192, 8192)]
ROWS = [96, 128, 256, 512, 1024, 2048]
ROUTES = ["hgemm", "fused", "library_tn", "hgemm_no_quarter"]   # (round 5: the last = hgemm without the 128 x 128 tile)


def timed(fn, reps=5):
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
    for N, K in WEIGHTS:
        W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
        del W
        for M in ROWS:
            X = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            def call(r):
                if r == "hgemm_no_quarter":
                    prev = F.lib.chgemm_set_quarter_tile(0, 0)
                    try:
                        F.gemm_4bit(X, q, st, out=out, _route="hgemm")
                    finally:
                        F.lib.chgemm_set_quarter_tile(prev, 0)
                else:
                    F.gemm_4bit(X, q, st, out=out, _route=r)
            for r in ROUTES:
                call(r)
            torch.cuda.synchronize()
            res = {r: [] for r in ROUTES}
            for _ in range(3):
                for r in ROUTES:
                    res[r].append(timed(lambda r=r: call(r)))
            med = {r: sorted(v)[1] for r, v in res.items()}
            best = min(med, key=med.get)
            print(f"{M:6d}x{N:6d}x{K:6d} static {F.gemm_4bit_static_route(M, N, K):7s} best {best:10s} " +
                  " ".join(f"{r} {med[r]:8.1f}" for r in ROUTES), flush=True)
            del X, out
        del q, st
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
