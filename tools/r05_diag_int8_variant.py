"""(Historical, round 6: chgemm_set_variant and the round-3 schedule arm it selected were removed from the library --
see DESIGN.md §2; this lab is kept as the record of the measurements it produced.)

Diagnostic: int8 igemmlt + dequant on the 4-wave k_hgemm, default schedule vs the round-3 arm (chgemm_set_variant(1)),
interleaved epilogue on / off, and the 8-wave igemm_256, at 4096 x 4096 x 11008: which pairs are bit-identical, how
many elements differ, and whether each arm is deterministic over repeats."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    m, n, k = 4096, 4096, 11008
    g = torch.Generator(device=dev).manual_seed(m + 3 * n + k)
    A = torch.randint(-127, 128, (m, k), device=dev, dtype=torch.int8, generator=g)
    B = torch.randint(-127, 128, (n, k), device=dev, dtype=torch.int8, generator=g)
    rs = torch.rand(m, device=dev, generator=g) * 2 + 0.5
    cs = torch.rand(n, device=dev, generator=g) * 2 + 0.5
    bias = torch.randn(n, device=dev, generator=g).half()
    arms = {"8w": (8, 0, 1), "4w v0 epi1": (4, 0, 1), "4w v0 epi0": (4, 0, 0), "4w v1": (4, 1, 1)}
    res = {}
    for name, (tile, v, epi) in arms.items():
        outs = []
        for _ in range(3):
            F.lib.cigemm_set_tile(tile)
            pv = F.lib.chgemm_set_variant(v)
            pe = F.lib.chgemm_set_epilogue(epi)
            try:
                outs.append(F.igemmlt_dequant(A, B, rs, cs, bias=bias).clone())
                torch.cuda.synchronize()
            finally:
                F.lib.chgemm_set_variant(pv)
                F.lib.chgemm_set_epilogue(pe)
                F.lib.cigemm_set_tile(0)
        det = all(torch.equal(outs[0], o) for o in outs[1:])
        res[name] = outs[0]
        print(f"{name}: deterministic over 3 runs: {det}", flush=True)
    ref = res["8w"]
    for name, o in res.items():
        d = (o != ref)
        idx = d.nonzero()
        print(f"{name} vs 8w: equal {torch.equal(o, ref)}  differing {int(d.sum())}  first {idx[:4].tolist()}", flush=True)
        if d.any():
            r, c = idx[0].tolist()
            print(f"   at {r},{c}: {float(o[r, c])} vs {float(ref[r, c])}; rows hit {sorted(set(idx[:, 0].tolist()))[:8]}"
                  f" cols mod 256 {sorted(set((idx[:, 1] % 256).tolist()))[:16]}", flush=True)


if __name__ == "__main__":
    main()
