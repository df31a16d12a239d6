"""Probe: does PyTorch TunableOp (hipBLASLt / rocBLAS solution search) beat the default heuristic for the
library GEMM of the NF4 metric shape (X[4096 x 11008] @ W[4096 x 11008]^T, bf16) and the 7B prefill shapes?
Writes the tuned table to gpurun_out/tunableop_results.csv.  Usage: python tools/tunableop_probe.py"""
import os

import torch

SHAPES = [(4096, 4096, 11008), (65536, 4096, 4096), (65536, 11008, 4096), (65536, 4096, 11008)]


def t_us(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


base = {}
ops = {}
for (m, n, k) in SHAPES:
    x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
    ops[(m, n, k)] = (x, w)
    base[(m, n, k)] = t_us(lambda: torch.matmul(x, w.t()))
    print(f"default  {m}x{n}x{k}: {base[(m, n, k)]:.1f} us  {2 * m * n * k / base[(m, n, k)] / 1e6:.0f} TF", flush=True)

os.makedirs("gpurun_out", exist_ok=True)
torch.cuda.tunable.enable(True)
torch.cuda.tunable.tuning_enable(True)
torch.cuda.tunable.set_max_tuning_duration(30)
torch.cuda.tunable.set_filename("gpurun_out/tunableop_results.csv")
for key, (x, w) in ops.items():
    torch.matmul(x, w.t())
    torch.cuda.synchronize()
    print("tuned", key, flush=True)
torch.cuda.tunable.tuning_enable(False)
for (m, n, k), (x, w) in ops.items():
    t = t_us(lambda: torch.matmul(x, w.t()))
    print(f"tunable  {m}x{n}x{k}: {t:.1f} us  {2 * m * n * k / t / 1e6:.0f} TF  ({base[(m, n, k)] / t:.3f}x)", flush=True)
torch.cuda.tunable.write_file()
