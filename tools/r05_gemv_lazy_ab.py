"""Round 5 A/B: the balanced decode GEMV's nested statistics decoded per chunk where consumed (cgemv_4bit_set_lazy_nested
1) against all before the first dot (0, round 4): config-2 weight 11008 x 4096 and the 70B 8-way decode shards, NF4
nested, bf16, 14 rotating copies (beyond the MALL), HIP-graph replay; outputs bit-identical.
Usage: python tools/r05_gemv_lazy_ab.py [rounds]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(2)
    for (n_out, k_in, copies) in [(11008, 4096, 14), (1280, 8192, 24), (7168, 8192, 8), (1024, 28672, 16)]:
        ws = []
        for _ in range(copies):
            W = (torch.randn(n_out, k_in, device=dev, generator=g) * 0.02).to(torch.bfloat16)
            ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
            del W
        x = torch.randn(1, k_in, device=dev, dtype=torch.bfloat16, generator=g)
        out = torch.empty(1, n_out, device=dev, dtype=torch.bfloat16)
        graphs, res = {}, {}
        for lazy in (0, 1):
            F.lib.cgemv_4bit_set_lazy_nested(lazy)
            for q, st in ws:
                F.gemv_4bit(x, q.t(), state=st, out=out)
            torch.cuda.synchronize()
            res[lazy] = out.clone()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for q, st in ws:
                    F.gemv_4bit(x, q.t(), state=st, out=out)
            graphs[lazy] = gr
        F.lib.cgemv_4bit_set_lazy_nested(1)
        ts = {0: [], 1: []}
        for _ in range(rounds):
            for lazy in (0, 1):
                graphs[lazy].replay()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    graphs[lazy].replay()
                e.record()
                e.synchronize()
                ts[lazy].append(s.elapsed_time(e) * 1e3 / 10 / copies)
        a, b = statistics.median(ts[0]), statistics.median(ts[1])
        print(f"gemv {n_out}x{k_in} nested: up front {a:6.2f} us   per chunk {b:6.2f} us   ({(b - a) / a * 100:+.1f} %)   "
              f"bitwise {torch.equal(res[0], res[1])}", flush=True)
        del graphs, ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
