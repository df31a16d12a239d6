"""A/B (GPU): the LLM.int8 inference forward at the metric shape (int8_row_quant of the 4096 x 11008 fp16 activations,
then the fused igemmlt + dequant) with the row quantise's int8 stores write-back vs write-through
(cint8_set_row_quant_store); HIP-graph replay, interleaved rounds after a clock ramp; outputs checked equal."""
import ctypes as ct
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import python_src_quants.functional as F  # noqa: E402
from python_src_quants.cextension import lib  # noqa: E402

M, N, K = 4096, 4096, 11008
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)
A = (torch.randn(M, K, device=dev, generator=g) * 2).half()
Wt = (torch.randn(N, K, device=dev, generator=g) * 0.05).half()
CB, _, SCB, _, _ = F.double_quant(Wt)
out = torch.empty(M, N, dtype=torch.float16, device=dev)
CA = torch.empty(M, K, dtype=torch.int8, device=dev)


def fwd():
    ca, sca = F.int8_row_quant(A, out_row=CA)
    F.igemmlt_dequant(ca, CB, sca, SCB, out=out)


def rq():
    F.int8_row_quant(A, out_row=CA)


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(reps):
            fn()
    gr.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        gr.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / (5 * reps)


refs = {}
for wt in (0, 1):
    lib.cint8_set_row_quant_store(ct.c_int(wt))
    CA.zero_()
    fwd()
    torch.cuda.synchronize()
    refs[wt] = (CA.clone(), out.clone())
assert torch.equal(refs[0][0], refs[1][0]) and torch.equal(refs[0][1], refs[1][1])
t0 = time.time()
while time.time() - t0 < 0.5:
    fwd()
torch.cuda.synchronize()
res = {0: {"rq": [], "fwd": []}, 1: {"rq": [], "fwd": []}}
for rnd in range(5):
    for wt in (0, 1):
        lib.cint8_set_row_quant_store(ct.c_int(wt))
        res[wt]["rq"].append(timed(rq))
        res[wt]["fwd"].append(timed(fwd))
lib.cint8_set_row_quant_store(ct.c_int(0))
for wt in (0, 1):
    print(f"row quantise stores {'write-through' if wt else 'write-back   '}: row quantise alone {sorted(res[wt]['rq'])[2]:6.2f} us"
          f"   row quantise + igemmlt+dequant {sorted(res[wt]['fwd'])[2]:7.2f} us", flush=True)
