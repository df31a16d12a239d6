"""A/B (GPU): the whole-K 32x32-MFMA few-token kernel (gemm4bit_fewtok.hip, cgemm_4bit_set_fewtok_mode(2)) against
the route gemm_4bit takes without it (mode 1: the multi-row GEMV at 2..4 rows, else the whole-K 16x16 kernel /
the split-K skinny kernel + reduce) and, at 1 row, against gemv_4bit.  Nested NF4 bs 64 (the Linear4bit default),
14 rotating weight copies per shape (> the 256 MB MALL for the big ones), HIP-graph replay, interleaved rounds,
medians; plus a max-|diff| check of every arm against dequantize_4bit + matmul in fp32.
Usage: python tools/fewtok32_ab.py [tokens ...]"""
import os
import sys
os.environ.setdefault("BNB_HIP_LIBRARY", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                   "bitsandbytes-sycl_amd", "build", "libbitsandbytes_hip_lab.so"))   # lab hooks: `make -C bitsandbytes-sycl_amd/csrc lab`

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bitsandbytes-sycl_amd"))
from python_src_quants import functional as F  # noqa: E402

TOKENS = [int(a) for a in os.environ.get("FT_TOKENS", "1,8,16,32").split(",")]
ABLS = [int(a) for a in sys.argv[1:]]
SHAPES = [tuple(int(v) for v in s.split("x")) for s in os.environ.get("FT_SHAPES", "11008x4096,4096x11008,4096x4096,14336x4096").split(",")]


def graph_time(calls, iters=20):
    for c in calls:
        c()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for c in calls:
            c()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters / len(calls)


def main():
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(3)
    for (n_out, k_in) in SHAPES:
        ws = []
        for _ in range(14):
            W = (torch.randn(n_out, k_in, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
            ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
            del W
        nbytes_w = n_out * k_in // 2 + n_out * k_in // 64 + n_out * k_in // 64 // 256 * 4
        Wd = F.dequantize_4bit(ws[0][0], ws[0][1]).float()
        for m in TOKENS:
            x = torch.randn(m, k_in, device=dev, dtype=torch.bfloat16, generator=gen)
            out = torch.empty(m, n_out, device=dev, dtype=torch.bfloat16)
            ref = x.float() @ Wd.t()
            rms = ref.pow(2).mean().sqrt().item()
            arms = [("fewtok", 2)] + [(f"abl{a}", 16 + a) for a in ABLS] + [("previous", 1)]
            if m == 1:
                arms.append(("gemv_4bit", -1))

            def calls_for(mode):
                if mode == -1:
                    return [(lambda q=q, st=st: F.gemv_4bit(x, q.t(), out=out, state=st)) for q, st in ws]
                # (mode -2: the multi-row GEMV, GEMM_4BIT_GEMV_TOKENS = 4 set by the caller)
                return [(lambda q=q, st=st: F.gemm_4bit(x, q, st, out=out)) for q, st in ws]
            if 2 <= m <= 4:
                arms.append(("tok_gemv", -2))
            res = {a: [] for a, _ in arms}
            err = {}
            for _ in range(5):
                for name, mode in arms:
                    F.GEMM_4BIT_GEMV_TOKENS = 4 if mode == -2 else 1
                    if mode == -2:
                        F.set_fewtok_mode(1)
                    elif mode >= 0:
                        F.set_fewtok_mode(mode)
                    res[name].append(graph_time(calls_for(mode)))
                    if name not in err:
                        calls_for(mode)[0]()
                        torch.cuda.synchronize()
                        err[name] = (out.float() - ref).abs().max().item() / rms
            F.set_fewtok_mode(0)
            nbytes = nbytes_w + m * k_in * 2 + m * n_out * 2
            line = f"{n_out}x{k_in} tokens {m:3d}:"
            for name, _ in arms:
                med = sorted(res[name])[2]
                line += f"  {name} {med:6.2f} us ({nbytes / med / 1e3:5.0f} GB/s, err {err[name]:.1e} rms)"
            print(line, flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
