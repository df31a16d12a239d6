"""Time the k_hgemm paths of whichever library BNB_HIP_LIBRARY names (round 6 A/B of hgemm.hip variant builds; run once
per library per round, rounds interleaved by the caller): the metric step (gemm_4bit NF4 4096 x 4096 x 11008: dequantise
+ k_hgemm), k_hgemm alone at that shape and at 4096^3, and the fused int8 igemmlt + dequant at both; us per call from
back-to-back launches after a clock ramp, with a checksum of each output so variants compare bit for bit."""
import ctypes as ct
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402

import python_src_quants.functional as F  # noqa: E402


def chk(t):
    b = t.contiguous().view(torch.int16 if t.element_size() == 2 else torch.int32).to(torch.int64).flatten()
    return int((b * torch.arange(1, b.numel() + 1, device=b.device, dtype=torch.int64)).sum().item())


def hgemm(a, w, c):
    F.pre_call(a.device)
    rc = F.lib.chgemm_tn_bf16(ct.c_int32(a.shape[0]), ct.c_int32(w.shape[0]), ct.c_int32(a.shape[1]), F.get_ptr(a),
                              ct.c_int32(a.stride(0)), F.get_ptr(w), ct.c_int32(w.stride(0)), F.get_ptr(c), ct.c_int32(c.stride(0)))
    assert rc == 0


def timed(fn, iters=50):
    t_end = time.time() + 0.3
    while time.time() < t_end:
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(11)
    res = {"lib": os.path.basename(os.environ.get("BNB_HIP_LIBRARY", "product"))}
    M, N, K = 4096, 4096, 11008
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
    W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    res["nf4_step"] = {"us": round(timed(lambda: F.gemm_4bit(X, q, st, out=Y)), 2), "checksum": chk(Y)}
    Wd = F.dequantize_4bit(q, st).contiguous()
    for (m, n, k) in ((4096, 4096, 11008), (4096, 4096, 4096)):
        a, w, c = X[:m, :k].contiguous(), Wd[:n, :k].contiguous(), torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        res[f"hgemm_{m}x{n}x{k}"] = {"us": round(timed(lambda: hgemm(a, w, c)), 2), "checksum": chk(c)}
        A8 = (torch.randn(m, k, device=dev, generator=g) * 2).half()
        W8 = (torch.randn(n, k, device=dev, generator=g) * 0.05).half()
        CA, _, SCA, _, _ = F.double_quant(A8)
        CB, _, SCB, _, _ = F.double_quant(W8)
        out = F.igemmlt_dequant(CA, CB, SCA, SCB)
        res[f"int8_{m}x{n}x{k}"] = {"us": round(timed(lambda: F.igemmlt_dequant(CA, CB, SCA, SCB, out=out)), 2),
                                     "checksum": chk(out)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
