"""Round 5 A/B: k_hgemm's C stores write-through (chgemm_set_c_store 1, the default) against write-through + the
non-temporal hint (2; the 256 x 256 tile's interleaved epilogue), interleaved rounds in one process: the metric step
(gemm_4bit = dequantise + k_hgemm at 4096 x 4096 x 11008, NF4 nested), bf16 k_hgemm alone at that shape, int8
igemmlt + fused mm_dequant at that shape and at 4096^3.  Outputs of both arms compared bit for bit.
Usage: python tools/r05_cstore_ab.py [rounds]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402


def timed(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    arms = []
    m, n, k = 4096, 4096, 11008
    W = (torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    X = torch.randn(m, k, device=dev, dtype=torch.bfloat16, generator=g)
    Y = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    arms.append(("metric step gemm_4bit", lambda: F.gemm_4bit(X, q, st, out=Y), Y))
    Y2 = torch.empty(m, n, device=dev, dtype=torch.bfloat16)

    def bf16():
        F.pre_call(dev)
        assert F.lib.chgemm_tn_bf16(m, n, k, F.get_ptr(X), k, F.get_ptr(W), k, F.get_ptr(Y2), n) == 0
    arms.append(("bf16 k_hgemm 4096x4096x11008", bf16, Y2))
    for (mm, nn, kk) in [(4096, 4096, 11008), (4096, 4096, 4096)]:
        A8 = torch.randint(-127, 128, (mm, kk), device=dev, dtype=torch.int8, generator=g)
        B8 = torch.randint(-127, 128, (nn, kk), device=dev, dtype=torch.int8, generator=g)
        rs = torch.rand(mm, device=dev, generator=g) * 2 + 0.5
        cs = torch.rand(nn, device=dev, generator=g) * 2 + 0.5
        bias = torch.randn(nn, device=dev, generator=g).half()
        O8 = torch.empty(mm, nn, device=dev, dtype=torch.float16)
        arms.append((f"int8 {mm}x{nn}x{kk}", lambda A8=A8, B8=B8, rs=rs, cs=cs, bias=bias, O8=O8:
                     F.igemmlt_dequant(A8, B8, rs, cs, bias=bias, out=O8), O8))
    for _ in range(20):
        arms[0][1]()
    torch.cuda.synchronize()
    for name, fn, out in arms:
        res = []
        for cst in (1, 2):
            F.lib.chgemm_set_c_store(cst)
            out.zero_()
            fn()
            torch.cuda.synchronize()
            res.append(out.clone())
        print(f"{name}: c_store 1 == 2 bitwise: {torch.equal(res[0], res[1])}", flush=True)
    times = {(name, c): [] for name, _, _ in arms for c in (1, 2)}
    for _ in range(rounds):
        for name, fn, _ in arms:
            for cst in (1, 2):
                F.lib.chgemm_set_c_store(cst)
                for _ in range(3):
                    fn()
                times[(name, cst)].append(timed(fn))
    F.lib.chgemm_set_c_store(1)
    for name, _, _ in arms:
        a, b = statistics.median(times[(name, 1)]), statistics.median(times[(name, 2)])
        print(f"{name}: write-through {a:7.1f} us   + non-temporal {b:7.1f} us   ({(b - a) / a * 100:+.1f} %)", flush=True)


if __name__ == "__main__":
    main()
