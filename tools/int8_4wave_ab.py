"""(Historical, round 6: chgemm_set_variant and the round-3 schedule arm it selected were removed from the library --
see DESIGN.md §2; this lab is kept as the record of the measurements it produced.)

A/B: the int8 igemmlt+dequant on the 4-wave kernel (hgemm.hip HG_I8_DEQ, forced by cigemm_set_tile(4)) against
the 8-wave igemm_256 (the default, cigemm_set_tile(0)), interleaved rounds in one process; bit-identity of the two outputs (both
are exact int32 + the same mm_dequant) and of the int32 products.  Usage: python tools/int8_4wave_ab.py [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    for (m, n, k) in ((4096, 4096, 11008), (4096, 4096, 4096), (65536 // 8, 11008, 4096)):
        g = torch.Generator(device=dev).manual_seed(3)
        A = torch.randint(-127, 128, (m, k), device=dev, dtype=torch.int8, generator=g)
        B = torch.randint(-127, 128, (n, k), device=dev, dtype=torch.int8, generator=g)
        rs = torch.rand(m, device=dev, generator=g) * 2 + 0.5
        cs = torch.rand(n, device=dev, generator=g) * 2 + 0.5
        bias = torch.randn(n, device=dev, generator=g).half()
        outs = {}
        for tile in (4, 0):
            F.lib.cigemm_set_tile(tile)
            outs[tile] = (F.igemmlt_dequant(A, B, rs, cs, bias=bias), F.igemm_rowmajor(A, B))
        F.lib.cigemm_set_tile(0)
        same = torch.equal(outs[4][0], outs[0][0]) and torch.equal(outs[4][1], outs[0][1])
        out = torch.empty(m, n, device=dev, dtype=torch.float16)
        times = {4: [], 0: []}
        for _ in range(rounds):
            for tile in (4, 0):
                F.lib.cigemm_set_tile(tile)
                for _ in range(3):
                    F.igemmlt_dequant(A, B, rs, cs, bias=bias, out=out)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    F.igemmlt_dequant(A, B, rs, cs, bias=bias, out=out)
                e.record()
                e.synchronize()
                times[tile].append(s.elapsed_time(e) / 20 * 1e3)
        F.lib.cigemm_set_tile(0)
        ops = 2.0 * m * n * k
        for tile, name in ((4, "4-wave (hgemm.hip)"), (0, "8-wave igemm_256")):
            t = sorted(times[tile])[len(times[tile]) // 2]
            print(f"{m}x{n}x{k} {name:22s} median {t:7.1f} us  min {min(times[tile]):7.1f}  {ops / t / 1e6:7.0f} TOPS")
        print(f"{m}x{n}x{k} bit-identical (fp16 dequant and int32): {same}", flush=True)


if __name__ == "__main__":
    main()
