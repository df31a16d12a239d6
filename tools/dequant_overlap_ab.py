"""A/B (GPU): the large-prefill library route at the metric shape (4096 x 4096 x 11008, NF4 bs 64) with the weight
dequantisation overlapped with the GEMM: the weight rows split in P parts, part p dequantised on a side stream while
the GEMM of part p-1 (torch.matmul into the output's column slice) runs on the main stream.  P = 1 is the serial
route.  Interleaved rounds, medians; max |difference| to P = 1 relative to its rms.
Usage: python tools/dequant_overlap_ab.py [P ...]"""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bitsandbytes-sycl_amd"))
from python_src_quants import functional as F  # noqa: E402

PARTS = [int(a) for a in sys.argv[1:]] or [1, 2, 4]
M, N, K, BS = 4096, 4096, 11008, 64


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
    W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=BS, quant_type="nf4", compress_statistics=True)
    del W
    am = F._absmax_fp32(st)
    Wd = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    side = torch.cuda.Stream()
    main_s = torch.cuda.current_stream()

    def deq(r0, r1):
        F.pre_call(dev)
        F.lib.cdequantize_blockwise_bf16_nf4(F.get_ptr(None), ct.c_void_p(q.data_ptr() + r0 * K // 2),
                                             ct.c_void_p(am.data_ptr() + 4 * (r0 * K // BS)),
                                             ct.c_void_p(Wd.data_ptr() + 2 * r0 * K), ct.c_int(BS), ct.c_int((r1 - r0) * K))

    def step(P):
        if P == 1:
            deq(0, N)
            torch.matmul(X, Wd.t(), out=out)
            return
        bounds = [N * p // P for p in range(P + 1)]
        side.wait_stream(main_s)              # the previous step's GEMMs have read Wd
        evs = []
        with torch.cuda.stream(side):
            for p in range(P):
                deq(bounds[p], bounds[p + 1])
                e = torch.cuda.Event()
                e.record(side)
                evs.append(e)
        for p in range(P):
            main_s.wait_event(evs[p])
            torch.matmul(X, Wd[bounds[p]:bounds[p + 1]].t(), out=out[:, bounds[p]:bounds[p + 1]])

    def t_us(P, it=20):
        step(P)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(it):
            step(P)
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) * 1e3 / it

    refs = {}
    for P in PARTS:
        step(P)
        torch.cuda.synchronize()
        refs[P] = out.float().clone()
    for _ in range(30):
        step(1)
    res = {P: [] for P in PARTS}
    for _ in range(7):
        for P in PARTS:
            res[P].append(t_us(P))
    rms = refs[PARTS[0]].pow(2).mean().sqrt().item()
    flops = 2.0 * M * N * K
    for P in PARTS:
        med = sorted(res[P])[3]
        d = (refs[P] - refs[PARTS[0]]).abs().max().item() / rms
        print(f"P={P}: {med:7.1f} us  {flops / med / 1e6:6.0f} TFLOP/s  (diff {d:.1e})", flush=True)


if __name__ == "__main__":
    main()
