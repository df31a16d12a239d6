"""Diagnostic: the tail-form side dequantise on the 128 x 128 tile (512 x 4096 x 4096, split-K 2): which outputs differ
from the plain k_hgemm launch, run to run."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402
from test_prefetch_gpu import _pf_gemm, _plain_gemm, _weight, _plan  # noqa: E402


def main():
    dtype = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(17)
    q2, s2 = _weight(11008, 4096, dtype, "nf4", True, 19)
    for rows, N, K in ((512, 4096, 4096), (256, 1024, 1024), (1024, 1024, 4096)):
        X = torch.randn(rows, K, device="cuda", generator=g).to(dtype)
        W = (torch.randn(N, K, device="cuda", generator=g) * 0.02).to(dtype)
        print("shape", rows, N, K, "plan", _plan(rows, N, K), flush=True)
        plain = [_plain_gemm(X, W) for _ in range(3)]
        torch.cuda.synchronize()
        print(" plain deterministic", all(torch.equal(plain[0], p) for p in plain[1:]), flush=True)
        ref = (X.float() @ W.float().t())
        for mode in (1, 129):
            F.lib.chgemm_set_side_mode(mode)
            outs = []
            for _ in range(3):
                o, nxt = _pf_gemm(X, W, (q2, s2))
                torch.cuda.synchronize()
                outs.append(o)
            d = outs[0] != plain[0]
            idx = d.nonzero()
            print(f" mode {mode}: pf deterministic {all(torch.equal(outs[0], o) for o in outs[1:])}, differs from plain "
                  f"{int(d.sum())}, max|pf-ref| {float((outs[0].float() - ref).abs().max()):.4f}, max|plain-ref| "
                  f"{float((plain[0].float() - ref).abs().max()):.4f}", flush=True)
            if d.any():
                print("   rows", sorted(set((idx[:, 0] % 128).tolist()))[:20], "cols", sorted(set((idx[:, 1] % 128).tolist()))[:20],
                      "tiles", sorted(set(((idx[:, 0] // 128) * 100 + idx[:, 1] // 128).tolist()))[:20], flush=True)
        F.lib.chgemm_set_side_mode(1)


if __name__ == "__main__":
    main()
