"""Probe: does PyTorch TunableOp (hipBLASLt / rocBLAS solution search) beat the default heuristic for the
library GEMM of the NF4 metric shape (X[4096 x 11008] @ W[4096 x 11008]^T, bf16) and the 7B prefill shapes?
Round 2b: the default is measured warm and interleaved with the tuned solution (TunableOp switched on and off
between rounds), so warm-up and clock drift hit both arms alike.  Writes the tuned table to
gpurun_out/tunableop_results.csv.  Usage: python tools/tunableop_probe.py [shape ...]  (shape = MxNxK)"""
import os
import sys
import time

import torch

SHAPES = [(4096, 4096, 11008), (2048, 4096, 11008), (4096, 11008, 4096), (65536, 4096, 11008)]
if len(sys.argv) > 1:
    SHAPES = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]]


def t_us(fn, it=30):
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


ops = {}
for (m, n, k) in SHAPES:
    x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
    ops[(m, n, k)] = (x, w)
# clock ramp on the default solutions
t_end = time.perf_counter() + 2.0
while time.perf_counter() < t_end:
    for (x, w) in ops.values():
        torch.matmul(x, w.t())
    torch.cuda.synchronize()

os.makedirs("gpurun_out", exist_ok=True)
torch.cuda.tunable.set_filename("gpurun_out/tunableop_results.csv")
torch.cuda.tunable.set_max_tuning_duration(30)
torch.cuda.tunable.enable(True)
torch.cuda.tunable.tuning_enable(True)
for key, (x, w) in ops.items():
    torch.matmul(x, w.t())
    torch.cuda.synchronize()
    print("tuned", key, flush=True)
torch.cuda.tunable.tuning_enable(False)

res = {key: {"default": [], "tuned": []} for key in ops}
for rnd in range(5):
    for arm in ("default", "tuned"):
        torch.cuda.tunable.enable(arm == "tuned")
        for key, (x, w) in ops.items():
            res[key][arm].append(t_us(lambda: torch.matmul(x, w.t())))
for (m, n, k), r in res.items():
    d = sorted(r["default"])[2]
    t = sorted(r["tuned"])[2]
    f = 2 * m * n * k
    print(f"{m}x{n}x{k}: default {d:.1f} us ({f / d / 1e6:.0f} TF)  tuned {t:.1f} us ({f / t / 1e6:.0f} TF)  "
          f"-> {d / t:.3f}x  (medians of 5 interleaved rounds)", flush=True)
torch.cuda.tunable.enable(True)     # the results file is written at exit
