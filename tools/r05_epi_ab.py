"""Round 5 A/B: k_hgemm's interleaved 16-bit epilogue (chgemm_set_epilogue 1, HG_V_EPI) against the round-4 one (0), on
the library's own entry points, interleaved rounds in one process: bf16 at the metric shape (4096 x 4096 x 11008) and
4096^3, int8 igemmlt + fused mm_dequant at the same two shapes.  Outputs of both arms compared bit for bit.  Also the
33..64-token path (11008 x 4096 NF4 nested at 33 / 64 rows, graph replay over 14 weight copies) as routed.
Usage: python tools/r05_epi_ab.py [rounds]"""
import os
import statistics
import sys
import time

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
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    arms = []
    for (m, n, k) in [(4096, 4096, 11008), (4096, 4096, 4096)]:
        X = torch.randn(m, k, device=dev, dtype=torch.bfloat16, generator=g)
        W = (torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        Y = torch.empty(m, n, device=dev, dtype=torch.bfloat16)

        def bf16(X=X, W=W, Y=Y, m=m, n=n, k=k):
            F.pre_call(dev)
            assert F.lib.chgemm_tn_bf16(m, n, k, F.get_ptr(X), k, F.get_ptr(W), k, F.get_ptr(Y), n) == 0
        A8 = torch.randint(-127, 128, (m, k), device=dev, dtype=torch.int8, generator=g)
        B8 = torch.randint(-127, 128, (n, k), device=dev, dtype=torch.int8, generator=g)
        rs = torch.rand(m, device=dev, generator=g) * 2 + 0.5
        cs = torch.rand(n, device=dev, generator=g) * 2 + 0.5
        bias = torch.randn(n, device=dev, generator=g).half()
        O8 = torch.empty(m, n, device=dev, dtype=torch.float16)
        i8 = lambda A8=A8, B8=B8, rs=rs, cs=cs, bias=bias, O8=O8: F.igemmlt_dequant(A8, B8, rs, cs, bias=bias, out=O8)  # noqa
        arms.append((f"bf16 {m}x{n}x{k}", bf16, Y))
        arms.append((f"int8 {m}x{n}x{k}", i8, O8))
    t_end = time.perf_counter() + 0.5
    while time.perf_counter() < t_end:
        arms[0][1]()
        torch.cuda.synchronize()
    for name, fn, out in arms:
        res = []
        for epi in (0, 1):
            F.lib.chgemm_set_epilogue(epi)
            out.zero_()
            fn()
            torch.cuda.synchronize()
            res.append(out.clone())
        print(f"{name}: epilogue 0 == 1 bitwise: {torch.equal(res[0], res[1])}", flush=True)
    times = {(name, epi): [] for name, _, _ in arms for epi in (0, 1)}
    for r in range(rounds):
        for name, fn, _ in arms:
            for epi in (0, 1):
                F.lib.chgemm_set_epilogue(epi)
                for _ in range(3):
                    fn()
                times[(name, epi)].append(timed(fn))
    F.lib.chgemm_set_epilogue(1)
    for name, _, _ in arms:
        a, b = statistics.median(times[(name, 0)]), statistics.median(times[(name, 1)])
        print(f"{name}: round-4 epilogue {a:7.1f} us   interleaved {b:7.1f} us   ({(b - a) / a * 100:+.1f} %)", flush=True)
    # the metric step's dequantise (4096 x 11008 NF4, nested statistics): per-lane vs scalar statistics loads, alone and
    # in the step (dequantise + k_hgemm, the bench's gemm_4bit call)
    import ctypes as ct
    gw = torch.Generator(device=dev).manual_seed(1000)
    Wm = (torch.randn(4096, 11008, device=dev, generator=gw) * 0.02).to(torch.bfloat16)
    qm, stm = F.quantize_4bit(Wm, blocksize=64, quant_type="nf4", compress_statistics=True)
    del Wm
    Xm = torch.randn(4096, 11008, device=dev, dtype=torch.bfloat16, generator=gw)
    Ym = torch.empty(4096, 4096, device=dev, dtype=torch.bfloat16)
    Wd = torch.empty(4096, 11008, device=dev, dtype=torch.bfloat16)
    deq = lambda: F._dequant_4bit_nested(qm, stm, Wd)  # noqa: E731
    step = lambda: F.gemm_4bit(Xm, qm, stm, out=Ym)  # noqa: E731
    outs = []
    for sq in (0, 1):
        F.lib.cdequantize_set_nested_scalar(ct.c_int(sq))
        deq()
        torch.cuda.synchronize()
        outs.append(Wd.clone())
    print(f"dequantise per-lane == scalar stats bitwise: {torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))}",
          flush=True)
    td = {0: [], 1: []}
    ts = {0: [], 1: []}
    for r in range(rounds):
        for sq in (0, 1):
            F.lib.cdequantize_set_nested_scalar(ct.c_int(sq))
            for _ in range(3):
                deq()
            td[sq].append(timed(deq))
            for _ in range(3):
                step()
            ts[sq].append(timed(step))
    F.lib.cdequantize_set_nested_scalar(ct.c_int(1))
    print(f"dequantise 4096x11008 nested: per-lane stats {statistics.median(td[0]):6.2f} us   scalar stats "
          f"{statistics.median(td[1]):6.2f} us   (back to back, same weight)", flush=True)
    print(f"metric step (gemm_4bit: dequantise + k_hgemm): per-lane stats {statistics.median(ts[0]):7.1f} us   scalar stats "
          f"{statistics.median(ts[1]):7.1f} us", flush=True)
    del Xm, Ym, Wd
    # the 33..64-token path as routed (t64 + the reduce launch), graph replay over 14 weight copies
    n_out, k_in = 11008, 4096
    ws = []
    for _ in range(14):
        W = (torch.randn(n_out, k_in, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
    for mrows in (33, 48, 64):
        x = torch.randn(mrows, k_in, device=dev, dtype=torch.bfloat16, generator=g)
        out = torch.empty(mrows, n_out, device=dev, dtype=torch.bfloat16)
        calls = [(lambda q=q, st=st: F.gemm_4bit(x, q, st, out=out)) for q, st in ws]
        graphs, res = {}, {}
        for waves in (1, 2):                      # t64: 4 waves (one per SIMD) / 8 waves (two per SIMD)
            F.lib.cgemm_4bit_set_t64_waves(ct.c_int(waves))
            for c in calls:
                c()
            torch.cuda.synchronize()
            res[waves] = out.clone()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for c in calls:
                    c()
            graphs[waves] = gr
        F.lib.cgemm_4bit_set_t64_waves(ct.c_int(1))
        e = res[1].float()
        ok = bool(((res[2].float() - e).abs() <= 1e-2 * e.pow(2).mean().sqrt() + 1e-2 * e.abs()).all())
        ts = {1: [], 2: []}
        for _ in range(5):
            for waves in (1, 2):
                graphs[waves].replay()
                ts[waves].append(timed(graphs[waves].replay, reps=10) / len(calls))
        print(f"gemm_4bit 11008x4096 nested, {mrows} rows (graph replay, 14 copies): t64 4 waves "
              f"{statistics.median(ts[1]):6.2f} us   8 waves {statistics.median(ts[2]):6.2f} us   (close: {ok})", flush=True)


if __name__ == "__main__":
    main()
