"""Round 5 A/B: the 33..64-token kernel's register-fed form (cgemm_4bit_set_t64_regfed 2) against the LDS-DMA form +
reduce launch (1; 4 waves and, up to 48 rows, 8 waves), gemm_4bit on 14 rotating NF4 nested weight copies (~315 MB,
defeats the MALL), HIP-graph replay, median of interleaved rounds.  Shapes: the config-2 weight 11008 x 4096 (the
bench's few-token leg) and 4096 x 11008, 4096 x 4096, 28672 x 8192 (70B MLP, 8 copies).
Usage: python tools/r05_t64r_ab.py [rounds]"""
import ctypes as ct
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402


def timed(fn, reps=10):
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
    g = torch.Generator(device=dev).manual_seed(3)
    F.lib.cgemm_4bit_set_t64_mode(ct.c_int(2))          # the 33..64-token kernel wherever it applies
    for (n_out, k_in, copies) in [(11008, 4096, 14), (4096, 11008, 14), (4096, 4096, 14), (28672, 8192, 4)]:
        ws = []
        for _ in range(copies):
            W = (torch.randn(n_out, k_in, device=dev, generator=g) * 0.02).to(torch.bfloat16)
            ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
            del W
        for mrows in (33, 48, 64):
            x = torch.randn(mrows, k_in, device=dev, dtype=torch.bfloat16, generator=g)
            out = torch.empty(mrows, n_out, device=dev, dtype=torch.bfloat16)
            arms = {"lds 4w": (1, 1), "lds 8w": (1, 2), "regfed": (2, 1)}
            graphs, res = {}, {}
            for name, (rf, waves) in arms.items():
                F.lib.cgemm_4bit_set_t64_regfed(ct.c_int(rf))
                F.lib.cgemm_4bit_set_t64_waves(ct.c_int(waves))
                calls = [(lambda q=q, st=st: F.gemm_4bit(x, q, st, out=out)) for q, st in ws]
                for c in calls:
                    c()
                torch.cuda.synchronize()
                res[name] = out.clone()
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr):
                    for c in calls:
                        c()
                graphs[name] = gr
            F.lib.cgemm_4bit_set_t64_regfed(ct.c_int(0))
            F.lib.cgemm_4bit_set_t64_waves(ct.c_int(0))
            e = res["lds 4w"].float()
            ok = bool(((res["regfed"].float() - e).abs() <= 1e-2 * e.pow(2).mean().sqrt() + 1e-2 * e.abs()).all())
            ts = {name: [] for name in arms}
            for _ in range(rounds):
                for name in arms:
                    graphs[name].replay()
                    ts[name].append(timed(graphs[name].replay) / copies)
            line = "   ".join(f"{name} {statistics.median(v):6.2f} us" for name, v in ts.items())
            print(f"{n_out}x{k_in} {mrows} rows: {line}   (regfed close to lds 4w: {ok})", flush=True)
            del graphs
        del ws
        torch.cuda.empty_cache()
    F.lib.cgemm_4bit_set_t64_mode(ct.c_int(0))


if __name__ == "__main__":
    main()
