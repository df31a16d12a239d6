"""A/B (round 6): the 33..64-token kernel's geometry -- waves per 48-row set (4 / 8) x split-K count (the rule / forced) --
on the config-2 weight (11008 x 4096, nested) and its transpose, 14 rotating weight copies replayed from a HIP graph (the
bench's few-token leg), interleaved rounds; every arm's output checked against the default arm within the GEMM tolerance.
Fewer splits halve the fp32 partials the kernel writes and the reduce launch reads back."""
import ctypes as ct
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402

import python_src_quants.functional as F  # noqa: E402

LIB = F.lib


def graph_us(calls, iters=30):
    for c in calls:
        c()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for c in calls:
            c()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters / len(calls) * 1e3


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    out = {}
    for n_out, k_in in ((11008, 4096), (4096, 11008)):
        ws = []
        for _ in range(14):
            W = (torch.randn(n_out, k_in, device=dev, generator=g) * 0.02).to(torch.bfloat16)
            ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
            del W
        for m in (40, 48, 56, 64):
            x = torch.randn(m, k_in, device=dev, dtype=torch.bfloat16, generator=g)
            y = torch.empty(m, n_out, device=dev, dtype=torch.bfloat16)
            arms = {"auto": (0, 0), "w4_rule": (1, 0), "w8_rule": (2, 0), "w8_ks2": (2, 2), "w8_ks3": (2, 3),
                    "w4_ks2": (1, 2), "w4_ks3": (1, 3)}
            res = {a: [] for a in arms}
            ref = None
            ok = {}
            for rnd in range(5):
                for a, (wv, ks) in arms.items():
                    pw = LIB.cgemm_4bit_set_t64_waves(ct.c_int(wv))
                    pk = LIB.cgemm_4bit_set_t64_splits(ct.c_int(ks))
                    try:
                        calls = [(lambda q=q, st=st: F.gemm_4bit(x, q, st, out=y)) for q, st in ws]
                        res[a].append(graph_us(calls))
                        if rnd == 0:
                            o = F.gemm_4bit(x, ws[0][0], ws[0][1]).float()
                            if ref is None:
                                ref = o
                            d = (o - ref).abs()
                            ok[a] = bool((d <= 2e-2 * ref.pow(2).mean().sqrt() + 2e-2 * ref.abs()).all())
                    finally:
                        LIB.cgemm_4bit_set_t64_waves(ct.c_int(pw))
                        LIB.cgemm_4bit_set_t64_splits(ct.c_int(pk))
            out[f"{n_out}x{k_in}@{m}"] = {a: round(statistics.median(v), 2) for a, v in res.items()}
            out[f"{n_out}x{k_in}@{m}"]["within_tolerance"] = ok
            print(json.dumps({f"{n_out}x{k_in}@{m}": out[f"{n_out}x{k_in}@{m}"]}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
