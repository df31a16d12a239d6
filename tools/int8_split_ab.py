"""A/B (GPU): the fused igemmlt + dequant on the column shards of the multi-GPU INT8 step (tokens x N/g x K,
metric shape 4096 x 4096 x 11008, g = 1/2/4/8, and the 2-chunk halves the overlapped step runs), with the int8
split-K (auto) against the unsplit 256-tile kernel (cigemm_set_splitk(1)); interleaved rounds, medians.
Usage: [INT8_ROWS=4096,2048 INT8_COLS=4096,2048,1024,512] python tools/int8_split_ab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bitsandbytes-sycl_amd"))
from python_src_quants import functional as F  # noqa: E402


def t_us(fn, it=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / it


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    K = 11008
    for m in [int(v) for v in os.environ.get("INT8_ROWS", "4096,2048").split(",")]:
        A = torch.randint(-127, 128, (m, K), device=dev, dtype=torch.int8, generator=g)
        rs = torch.rand(m, device=dev, generator=g) + 0.5
        for n in [int(v) for v in os.environ.get("INT8_COLS", "4096,2048,1024,512").split(",")]:
            B = torch.randint(-127, 128, (n, K), device=dev, dtype=torch.int8, generator=g)
            cs = torch.rand(n, device=dev, generator=g) + 0.5
            out = torch.empty(m, n, device=dev, dtype=torch.float16)
            fn = lambda: F.igemmlt_dequant(A, B, rs, cs, out=out)  # noqa: E731
            res = {-1: [], 1: []}
            for _ in range(5):
                for ks in (-1, 1):
                    F.lib.cigemm_set_splitk(ks)
                    res[ks].append(t_us(fn))
            F.lib.cigemm_set_splitk(-1)
            ops = 2.0 * m * n * K
            a, b = sorted(res[-1])[2], sorted(res[1])[2]
            print(f"{m}x{n}x{K}: split-K(auto, bytes {F.lib.cigemmlt_workspace_bytes(m, n, K)}) {a:7.1f} us "
                  f"({ops / a / 1e6:5.0f} TOPS)   unsplit {b:7.1f} us ({ops / b / 1e6:5.0f} TOPS)", flush=True)


if __name__ == "__main__":
    main()
