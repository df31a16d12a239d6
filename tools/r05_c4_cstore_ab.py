"""Round 5 A/B: k_hgemm's C-store policy on multi-wave tile grids -- write-through (chgemm_set_c_store 1, default) vs
write-back (0) -- on the C4 layer (the seven Llama-2-7B NF4 projections at 65,536 tokens through gemm_4bit, as
bench.py times it) and per projection shape.  With 16-43 tiles per CU a write-back epilogue can land in the XCD's L2
and drain while the next tile computes; at one tile per CU (the metric shape) write-through won (round 4).
Usage: python tools/r05_c4_cstore_ab.py [rounds]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402


def timed(fn, reps=3):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(6)
    tokens, hid, inter = 65536, 4096, 11008
    shapes = [(hid, hid)] * 4 + [(inter, hid)] * 2 + [(hid, inter)]
    ws = []
    for n_out, k_in in shapes:
        W = (torch.randn(n_out, k_in, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
        del W
    X = torch.randn(tokens, hid, device=dev, dtype=torch.bfloat16, generator=g)
    Xi = torch.randn(tokens, inter, device=dev, dtype=torch.bfloat16, generator=g)
    outs = {n: torch.empty(tokens, n, device=dev, dtype=torch.bfloat16) for n in (hid, inter)}

    def proj(i):
        (n_out, k_in), (q, st) = shapes[i], ws[i]
        return lambda: F.gemm_4bit(X if k_in == hid else Xi, q, st, out=outs[n_out])

    def layer():
        for i in range(len(shapes)):
            proj(i)()
    res = {}
    for cst in (1, 0):
        F.lib.chgemm_set_c_store(cst)
        layer()
        torch.cuda.synchronize()
        res[cst] = [outs[hid].clone(), outs[inter].clone()]
    print(f"write-back == write-through bitwise: {all(torch.equal(a, b) for a, b in zip(res[0], res[1]))}", flush=True)
    del res
    arms = {"layer": layer, "q 4096x4096": proj(0), "gate 11008x4096": proj(4), "down 4096x11008": proj(6)}
    t = {(a, c): [] for a in arms for c in (1, 0)}
    for _ in range(rounds):
        for a, fn in arms.items():
            for cst in (1, 0):
                F.lib.chgemm_set_c_store(cst)
                fn()
                t[(a, cst)].append(timed(fn, 2 if a == "layer" else 5))
    F.lib.chgemm_set_c_store(1)
    for a in arms:
        wt, wb = statistics.median(t[(a, 1)]), statistics.median(t[(a, 0)])
        print(f"{a:18s}: write-through {wt:9.1f} us   write-back {wb:9.1f} us   ({(wb - wt) / wt * 100:+.1f} %)", flush=True)


if __name__ == "__main__":
    main()
