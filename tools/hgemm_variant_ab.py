"""(Historical, round 6: chgemm_set_variant and the round-3 schedule arm it selected were removed from the library --
see DESIGN.md §2; this lab is kept as the record of the measurements it produced.)

A/B of the k_hgemm schedules (chgemm_set_variant 0 = default, 1 = the alternative arm) on the library's own entry
points, interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24): bf16 chgemm_tn at the metric shape
and the int8 igemmlt + dequant on the 4-wave body (cigemm_set_tile(4)) against the 8-wave igemm_256 (tile 8).  Outputs
of every arm are compared bit for bit.  Usage: python tools/hgemm_variant_ab.py [rounds]"""
import ctypes as ct
import os
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
    shapes = [(4096, 4096, 11008), (4096, 4096, 4096)]
    arms = {}
    for (m, n, k) in shapes:
        X = torch.randn(m, k, device=dev, dtype=torch.bfloat16, generator=g)
        W = (torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        Y = torch.empty(m, n, device=dev, dtype=torch.bfloat16)

        def bf16(X=X, W=W, Y=Y, m=m, n=n, k=k):
            F.pre_call(dev)
            rc = F.lib.chgemm_tn_bf16(m, n, k, F.get_ptr(X), k, F.get_ptr(W), k, F.get_ptr(Y), n)
            assert rc == 0
        A8 = torch.randint(-127, 128, (m, k), device=dev, dtype=torch.int8, generator=g)
        B8 = torch.randint(-127, 128, (n, k), device=dev, dtype=torch.int8, generator=g)
        rs = torch.rand(m, device=dev, generator=g) * 2 + 0.5
        cs = torch.rand(n, device=dev, generator=g) * 2 + 0.5
        bias = torch.randn(n, device=dev, generator=g).half()
        O8 = torch.empty(m, n, device=dev, dtype=torch.float16)
        i8 = lambda A8=A8, B8=B8, rs=rs, cs=cs, bias=bias, O8=O8: F.igemmlt_dequant(A8, B8, rs, cs, bias=bias, out=O8)  # noqa
        arms[(m, n, k)] = [("bf16 v0", 0, None, bf16, Y), ("bf16 v1", 1, None, bf16, Y),
                           ("i8 4w v0", 0, 4, i8, O8), ("i8 4w v1", 1, 4, i8, O8), ("i8 8w", 0, 8, i8, O8)]
    # clock ramp
    t_end = time.perf_counter() + 0.5
    while time.perf_counter() < t_end:
        for sh in shapes:
            for _, v, tile, fn, _ in arms[sh][:1]:
                fn()
        torch.cuda.synchronize()
    for sh in shapes:
        outs = {}
        for name, v, tile, fn, out in arms[sh]:
            F.lib.chgemm_set_variant(v)
            if tile is not None:
                F.lib.cigemm_set_tile(tile)
            fn()
            torch.cuda.synchronize()
            outs[name] = out.clone()
        F.lib.chgemm_set_variant(0)
        F.lib.cigemm_set_tile(0)
        print(f"{sh} bf16 v0 == v1: {torch.equal(outs['bf16 v0'], outs['bf16 v1'])}; int8 4w v0 == v1 == 8w: "
              f"{torch.equal(outs['i8 4w v0'], outs['i8 4w v1']) and torch.equal(outs['i8 4w v0'], outs['i8 8w'])}")
    for r in range(rounds):
        for sh in shapes:
            line = []
            for name, v, tile, fn, _ in arms[sh]:
                F.lib.chgemm_set_variant(v)
                if tile is not None:
                    F.lib.cigemm_set_tile(tile)
                for _ in range(3):
                    fn()
                line.append(f"{name} {timed(fn):7.1f}")
            F.lib.chgemm_set_variant(0)
            F.lib.cigemm_set_tile(0)
            print(f"round {r} {sh}: " + " | ".join(line), flush=True)


if __name__ == "__main__":
    main()
