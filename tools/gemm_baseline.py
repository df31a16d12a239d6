"""Library baselines for the NF4 GEMM at the metric shape: the reference's own M>1 algorithm on the GPU
(dequantize_4bit -> bf16 F.linear, i.e. our dequant kernel + hipBLASLt) against the fused kernel, and
the bare bf16 GEMM (torch.matmul / F.linear on hipBLASLt) as the MFMA ceiling a library reaches here.
Usage (GPU box): python tools/gemm_baseline.py [M N K]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bitsandbytes-sycl_amd"))
import torch  # noqa: E402
import torch.nn.functional as tF  # noqa: E402

import python_src_quants.functional as F  # noqa: E402


def timeit(fn, iters=30, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3    # us


def sweep():
    """fused kernel vs dequantise + matmul over (tokens, features) at K = 11008 (multi-GPU shard shapes)"""
    dev = torch.device("cuda:0")
    K = 11008
    g = torch.Generator(device=dev).manual_seed(0)
    for N in (512, 1024, 2048, 4096):
        W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
        am = F._absmax_fp32(st)
        Wd = torch.empty_like(W)
        for M in (256, 512, 1024, 2048, 4096):
            X = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
            Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            t_f = timeit(lambda: F.gemm_4bit(X, q, st, out=Y, absmax=am, _route="fused"))
            t_l = timeit(lambda: F.gemm_4bit(X, q, st, out=Y, absmax=am, _route="library"))
            t_d = timeit(lambda: F.dequantize_4bit(q, st, out=Wd))
            print(f"N={N:5d} M={M:5d}  fused {t_f:8.1f} us   dequant+matmul {t_l:8.1f} us   (dequant alone {t_d:6.1f})",
                  flush=True)


def int8():
    """igemmlt (fused int32 -> fp16 mm_dequant) vs torch._int_mm (hipBLASLt int8) at the metric shapes"""
    dev = torch.device("cuda:0")
    for M, N, K in ((4096, 4096, 11008), (4096, 4096, 4096)):
        g = torch.Generator(device=dev).manual_seed(3)
        A = (torch.randn(M, K, device=dev, generator=g) * 2).half()
        Wt = (torch.randn(N, K, device=dev, generator=g) * 0.05).half()
        CB, _, SCB, _, _ = F.double_quant(Wt)
        CA, _, SCA, _, _ = F.double_quant(A)
        out = torch.empty(M, N, dtype=torch.float16, device=dev)
        ops = 2.0 * M * N * K
        t = timeit(lambda: F.igemmlt_dequant(CA, CB, SCA, SCB, out=out))
        print(f"{M}x{N}x{K} igemmlt+dequant (ours)   {t:8.1f} us  {ops / t / 1e6:8.1f} TOPS", flush=True)
        try:
            t2 = timeit(lambda: torch._int_mm(CA, CB.t()))
            print(f"{M}x{N}x{K} torch._int_mm (library) {t2:8.1f} us  {ops / t2 / 1e6:8.1f} TOPS", flush=True)
        except Exception as ex:  # noqa: BLE001
            print("torch._int_mm failed:", ex)
        t_st = timeit(lambda: F.get_colrow_absmax(A))
        rs_, cs_, _ = F.get_colrow_absmax(A)
        t_dq = timeit(lambda: F.double_quant(A, col_stats=cs_, row_stats=rs_))
        t_full = timeit(lambda: F.double_quant(A))

        def fwd():
            ca, _, sca, _, _ = F.double_quant(A)
            F.igemmlt_dequant(ca, CB, sca, SCB, out=out)
        t_fwd = timeit(fwd)
        print(f"  colrow_stats {t_st:.1f} us, rowcol_quant {t_dq:.1f} us, double_quant {t_full:.1f} us, "
              f"forward {t_fwd:.1f} us", flush=True)
        t3 = timeit(lambda: torch.matmul(A, Wt.t()))
        print(f"{M}x{N}x{K} fp16 matmul (library)   {t3:8.1f} us  {ops / t3 / 1e6:8.1f} TFLOP/s", flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "sweep":
        return sweep()
    if len(sys.argv) > 1 and sys.argv[1] == "int8":
        return int8()
    M, N, K = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (4096, 4096, 11008)
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    flop = 2.0 * M * N * K
    Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    res = {}
    res["fused gemm_4bit"] = timeit(lambda: F.gemm_4bit(X, q, st, out=Y))
    res["bf16 F.linear (hipBLASLt)"] = timeit(lambda: tF.linear(X, W))
    res["bf16 torch.matmul X @ W.T"] = timeit(lambda: torch.matmul(X, W.t()))
    Wd = torch.empty_like(W)
    res["dequantize_4bit only"] = timeit(lambda: F.dequantize_4bit(q, st, out=Wd))
    res["dequantize_4bit + F.linear"] = timeit(lambda: tF.linear(X, F.dequantize_4bit(q, st, out=Wd)))
    # dequant of N-chunk c+1 on a side stream while hipBLASLt runs chunk c
    side = torch.cuda.Stream(device=dev)
    main_s = torch.cuda.current_stream(dev)
    for chunks in (2, 4, 8):
        nc = N // chunks
        Wc = [torch.empty(nc, K, device=dev, dtype=torch.bfloat16) for _ in range(2)]
        qs = [F.quantize_4bit(W[c * nc:(c + 1) * nc], blocksize=64, quant_type="nf4", compress_statistics=True)
              for c in range(chunks)]
        evs = [torch.cuda.Event() for _ in range(chunks)]
        Yc = [torch.empty(M, nc, device=dev, dtype=torch.bfloat16) for _ in range(chunks)]   # column blocks

        def run():
            side.wait_stream(main_s)
            with torch.cuda.stream(side):
                F.dequantize_4bit(qs[0][0], qs[0][1], out=Wc[0])
                evs[0].record(side)
            for c in range(chunks):
                main_s.wait_event(evs[c])
                if c + 1 < chunks:
                    with torch.cuda.stream(side):
                        side.wait_stream(main_s) if c >= 1 else None
                        F.dequantize_4bit(qs[c + 1][0], qs[c + 1][1], out=Wc[(c + 1) % 2])
                        evs[c + 1].record(side)
                torch.matmul(X, Wc[c % 2].t(), out=Yc[c])
        res[f"dequant||matmul, {chunks} N-chunks"] = timeit(run)
    for k, us in res.items():
        print(f"{k:32s} {us:9.1f} us  {flop / us / 1e6:8.1f} TFLOP/s")
    for m in (16, 64, 256, 512, 1024, 2048):
        Xm = X[:m]
        Ym = torch.empty(m, N, device=dev, dtype=torch.bfloat16)
        t_f = timeit(lambda: F.gemm_4bit(Xm, q, st, out=Ym))
        t_l = timeit(lambda: tF.linear(Xm, F.dequantize_4bit(q, st, out=Wd)))
        print(f"M={m:5d}  fused {t_f:8.1f} us   dequant+linear {t_l:8.1f} us")


if __name__ == "__main__":
    main()
