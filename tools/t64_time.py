"""Time the few-token GEMM on the config-2 weight (11008 x 4096 NF4 nested, bf16) at 33..64 rows: the new kernel
(gemm4bit_t64.hip) vs the split-K weight-stream kernel it replaces (cgemm_4bit_set_t64_mode(1)), HIP-graph replay over
14 rotating weight copies (past the MALL), like bench.py's few-token leg."""
import ctypes as ct
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import python_src_quants.functional as F  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda", 0)
# arm -> (t64 mode, in-kernel combine, partial-store policy)
ARMS = {"t64": (0, 0, 0), "t64_pstore_wt_dword": (0, 0, 1), "t64_pstore_wt_lines": (0, 0, 2),
        "t64_combine": (0, 1, 0), "skinny": (1, 0, 0)}
shapes = [(11008, 4096), (4096, 11008), (4096, 4096)]
for N, K in shapes:
    g = torch.Generator(device=dev).manual_seed(1)
    copies = []
    for _ in range(14 if N * K > 20_000_000 else 30):
        W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        copies.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
    for M in (33, 48, 64):
        X = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
        outs = [torch.empty(M, N, device=dev, dtype=torch.bfloat16) for _ in copies]
        res = {}
        for rnd in range(3):                                  # interleaved rounds, median
            for arm, (mode, comb, ps) in ARMS.items():
                F.lib.cgemm_4bit_set_t64_mode(ct.c_int(mode))
                F.lib.cgemm_4bit_set_t64_combine(ct.c_int(comb))
                F.lib.cgemm_4bit_set_t64_pstore(ct.c_int(ps))
                calls = [(lambda q=q, s=s, o=o: F.gemm_4bit(X, q, s, out=o)) for (q, s), o in zip(copies, outs)]
                res.setdefault(arm, []).append(bench._time_graph(calls, 10) * 1e6)
        F.lib.cgemm_4bit_set_t64_mode(ct.c_int(0))
        F.lib.cgemm_4bit_set_t64_combine(ct.c_int(0))
        F.lib.cgemm_4bit_set_t64_pstore(ct.c_int(0))
        med = {a: sorted(v)[1] for a, v in res.items()}
        print(f"{N}x{K} rows {M}: " + "   ".join(f"{a} {v:.2f} us" for a, v in med.items()), flush=True)
