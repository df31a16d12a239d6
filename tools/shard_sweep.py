"""Per-rank GEMM time of the column-sharded NF4 metric shape (M=4096, K=11008, N/g rows of W) for each
tile kernel: which kernel should a shard of width N/g use.  Usage: python tools/shard_sweep.py"""
import os
import sys
import ctypes as ct

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402
from python_src_quants.cextension import lib  # noqa: E402

dev = torch.device("cuda", 0)
K = 11008
Xall = torch.randn(4096, K, device=dev, dtype=torch.bfloat16)
for M, n in ((4096, 4096), (4096, 2048), (2048, 2048), (4096, 1024), (2048, 1024), (1024, 1024), (4096, 512),
             (2048, 512), (1024, 512)):
    X = Xall[:M]
    W = (torch.randn(n, K, device=dev) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=False)
    Y = torch.empty(M, n, device=dev, dtype=torch.bfloat16)
    for tile in sys.argv[1:] and [int(a) for a in sys.argv[1:]] or (128, 256, 0):
        lib.cgemm_4bit_set_tile(ct.c_int(tile))
        for _ in range(3):
            F.gemm_4bit(X, q, st, out=Y)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        R = 20
        for _ in range(R):
            F.gemm_4bit(X, q, st, out=Y)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / R * 1e3
        print(f"M={M:5d} N={n:5d} tile={tile:3d}  {us:8.1f} us  {2.0 * M * n * K / us / 1e6:7.1f} TFLOP/s", flush=True)
    lib.cgemm_4bit_set_tile(ct.c_int(0))
