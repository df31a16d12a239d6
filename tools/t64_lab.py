"""Ablations of the 33..64-token kernel (cgemm_4bit_set_t64_mode 16 + ABL; timing only, wrong results) at 11008 x 4096,
64 rows, nested NF4, bf16; HIP-graph replay over 14 rotating weight copies.  Mode 15: the kernel without its reduce."""
import ctypes as ct
import os
import sys
os.environ.setdefault("BNB_HIP_LIBRARY", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                   "bitsandbytes-sycl_amd", "build", "libbitsandbytes_hip_lab.so"))   # lab hooks: `make -C bitsandbytes-sycl_amd/csrc lab`

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import python_src_quants.functional as F  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda", 0)
N, K, M = 11008, 4096, 64
g = torch.Generator(device=dev).manual_seed(1)
copies = []
for _ in range(14):
    W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    copies.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
X = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
outs = [torch.empty(M, N, device=dev, dtype=torch.bfloat16) for _ in copies]
names = {0: "full", 15: "no reduce", 17: "no vmcnt waits", 22: "no token + weight DMA", 40: "no MFMA + lookups",
         48: "no output stores (computed)", 80: "no table build", 144: "no loop barriers",
         (0, 1): "1 split", (0, 2): "2 splits", (0, 3): "3 splits", (0, 6): "6 splits", (15, 2): "2 splits, no reduce",
         1: "previous kernel (skinny)"}
for rnd in range(2):
    for mode, name in names.items():
        ks = 0
        if isinstance(mode, tuple):
            mode, ks = mode
        F.lib.cgemm_4bit_set_t64_splits(ct.c_int(ks))
        F.lib.cgemm_4bit_set_t64_mode(ct.c_int(mode))
        calls = [(lambda q=q, s=s, o=o: F.gemm_4bit(X, q, s, out=o)) for (q, s), o in zip(copies, outs)]
        t = bench._time_graph(calls, 10) * 1e6
        if rnd == 1:
            print(f"{name:24s} {t:7.2f} us")
F.lib.cgemm_4bit_set_t64_mode(ct.c_int(0))
F.lib.cgemm_4bit_set_t64_splits(ct.c_int(0))
