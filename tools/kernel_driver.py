"""Run one hot-path kernel repeatedly (for rocprofv3 counter passes / A-B timing on the GPU box).
Usage: python tools/kernel_driver.py {nf4gemm,int8gemm,gemv,dequant} [iters]"""
import ctypes as ct
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402


def main():
    what = sys.argv[1]
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    if what == "nf4gemm":
        M, N, K = 4096, 4096, 11008
        X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4")
        Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fn = lambda: F.gemm_4bit(X, q, st, out=Y, absmax=st.absmax)  # noqa: E731
        flops = 2.0 * M * N * K
    elif what == "int8gemm":
        M, N, K = 4096, 4096, 11008
        A = torch.randint(-127, 128, (M, K), device=dev, dtype=torch.int8)
        B = torch.randint(-127, 128, (N, K), device=dev, dtype=torch.int8)
        rs = torch.rand(M, device=dev) + 0.5
        cs = torch.rand(N, device=dev) + 0.5
        out = torch.empty(M, N, device=dev, dtype=torch.float16)
        fn = lambda: F.igemmlt_dequant(A, B, rs, cs, out=out)  # noqa: E731
        flops = 2.0 * M * N * K
    elif what in ("gemv", "gemv16", "gemvn"):
        # decode: M=1, N=11008, K=4096, 14 rotating weight copies (> MALL) replayed from one HIP graph
        dt = torch.bfloat16 if what == "gemv" else torch.float16
        n_out, k_in, copies = 11008, 4096, 14
        ws = []
        for _ in range(copies):
            W = (torch.randn(n_out, k_in, device=dev) * 0.02).to(dt)
            ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=(what == "gemvn")))
        x = torch.randn(1, k_in, device=dev, dtype=dt)
        out = torch.empty(1, n_out, device=dev, dtype=dt)
        for q, st in ws:
            F.gemv_4bit(x, q.t(), out=out, state=st)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for q, st in ws:
                F.gemv_4bit(x, q.t(), out=out, state=st)
        fn = g.replay
        iters_per = copies
        nbytes = n_out * k_in // 2 + n_out * k_in // 64 * 4 + k_in * 2 + n_out * 2
        if what == "gemvn":   # 1-B codes + fp32 per 256 blocks + 1 KiB code map
            nbytes = n_out * k_in // 2 + n_out * k_in // 64 + n_out * k_in // 64 // 256 * 4 + 1024 + k_in * 2 + n_out * 2
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / iters / iters_per * 1e-3
        print(f"{what}: {t*1e6:.2f} us/call (graph), {nbytes / t / 1e9:.0f} GB/s")
        return
    elif what == "dequant":
        # config 1 on the GPU: NF4 4096x4096 bs=64 -> bf16, 30 rotating copies, one HIP graph
        copies = 30
        qs = [F.quantize_4bit(torch.randn(4096, 4096, device=dev), blocksize=64, quant_type="nf4") for _ in range(copies)]
        outs = [torch.empty(4096, 4096, device=dev, dtype=torch.bfloat16) for _ in range(2)]

        def call(q, st, o):
            F.pre_call(dev)
            F.lib.cdequantize_blockwise_bf16_nf4(None, F.get_ptr(q), F.get_ptr(st.absmax), F.get_ptr(o),
                                                 ct.c_int(64), ct.c_int(4096 * 4096))
        for i, (q, st) in enumerate(qs):
            call(q, st, outs[i % 2])
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i, (q, st) in enumerate(qs):
                call(q, st, outs[i % 2])
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            g.replay()
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / iters / copies * 1e-3
        print(f"dequant: {t*1e6:.2f} us/call (graph), {42991616 / t / 1e9:.0f} GB/s")
        return
    elif what == "nf4gemm_rand":   # uniform random packed bytes / absmax 0.01 (the lab's data)
        M, N, K = 4096, 4096, 11008
        X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4")
        q.copy_(torch.randint(0, 256, q.shape, device=dev, dtype=torch.uint8))
        st.absmax.fill_(0.01)
        Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fn = lambda: F.gemm_4bit(X, q, st, out=Y, absmax=st.absmax)  # noqa: E731
        flops = 2.0 * M * N * K
    else:
        raise SystemExit(f"unknown {what}")
    for _ in range(int(os.environ.get("KD_WARMUP", "3"))):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    t = s.elapsed_time(e) / iters * 1e-3
    print(f"{what}: {t*1e6:.1f} us/call, {flops / t / 1e12:.1f} T(FL)OP/s")


if __name__ == "__main__":
    main()
