"""Probe: hipBLASLt int8 GEMM (torch._int_mm) at the igemmlt metric shapes, for comparison with k_igemm_256.

Timing: CUDA events over 50 launches after 10 warmups; prints TOPS.  Used as a ceiling reference only.
"""
import torch

for (m, n, k) in [(4096, 4096, 11008), (4096, 4096, 4096)]:
    a = torch.randint(-127, 128, (m, k), dtype=torch.int8, device="cuda")
    b = torch.randint(-127, 128, (n, k), dtype=torch.int8, device="cuda")
    for name, fn in [("A @ B^T (B row-major NxK)", lambda: torch._int_mm(a, b.t())),
                     ("A @ Bkn (B contiguous KxN)", (lambda bt: (lambda: torch._int_mm(a, bt)))(b.t().contiguous()))]:
        try:
            for _ in range(10):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            for _ in range(50):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 50
            print(f"{m}x{n}x{k} {name}: {us:.1f} us  {2 * m * n * k / us / 1e6:.0f} TOPS", flush=True)
        except Exception as ex:   # noqa: BLE001 - probe prints whatever the library refuses
            print(f"{m}x{n}x{k} {name}: failed: {ex}", flush=True)
