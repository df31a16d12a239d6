"""Round 5 A/B: the 128 x 128 k_hgemm tile (chgemm_set_quarter_tile) on the shapes that run split-K or half-empty grids
today -- the rank shards of the multi-GPU metric step and of the 70B layer -- against the current plans: mode 0 (never),
forced (2), with the plan each takes; bf16 through chgemm_tn_ws_bf16 with the plan's workspace, median of 5 rounds of
10 launches.  Unsplit plans of both tiles must give the same bits (same MFMA sequence per output block).
Usage: python tools/r05_quarter_tile_ab.py"""
import ctypes as ct
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402

dev = torch.device("cuda", 0)
SHAPES = [(4096, 128, 8192), (4096, 512, 11008), (2048, 512, 11008), (4096, 1024, 8192), (4096, 1024, 11008),
          (4096, 1024, 28672), (2048, 1024, 11008), (4096, 1280, 8192), (4096, 2048, 11008), (4096, 3584, 8192),
          (4096, 7168, 8192), (1024, 4096, 4096), (512, 4096, 11008), (256, 11008, 4096), (4096, 4096, 11008)]


def plan(m, n, k):
    o = (ct.c_int * 4)()
    F.lib.chgemm_tn_plan(m, n, k, o)
    return tuple(o)


def run(X, W, Y, m, n, k, ws, nbytes):
    F.pre_call(dev)
    rc = F.lib.chgemm_tn_ws_bf16(m, n, k, F.get_ptr(X), k, F.get_ptr(W), k, F.get_ptr(Y), n, F.get_ptr(ws),
                                 ct.c_longlong(nbytes))
    assert rc == 0


def timed(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    g = torch.Generator(device=dev).manual_seed(5)
    ws = torch.empty(256 << 20, dtype=torch.float32, device=dev)   # 1 GiB: every plan's partials fit
    for (m, n, k) in SHAPES:
        X = (torch.rand(m, k, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        W = (torch.rand(n, k, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        Y = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        res, plans, ts = {}, {}, {}
        for mode in (0, 2, 1):
            F.lib.chgemm_set_quarter_tile(mode, 0)
            plans[mode] = plan(m, n, k)
            fn = lambda: run(X, W, Y, m, n, k, ws, ws.numel() * 4)  # noqa: E731
            fn()
            torch.cuda.synchronize()
            res[mode] = Y.clone()
            ts[mode] = []
        for _ in range(5):
            for mode in (0, 2, 1):
                F.lib.chgemm_set_quarter_tile(mode, 0)
                fn = lambda: run(X, W, Y, m, n, k, ws, ws.numel() * 4)  # noqa: E731
                fn()
                ts[mode].append(timed(fn))
        F.lib.chgemm_set_quarter_tile(1, 0)
        same = ""
        if plans[0][2] == 1 and plans[2][2] == 1:
            same = f"  unsplit bits equal: {torch.equal(res[0], res[2])}"
        e = res[0].float()
        close = bool(((res[2].float() - e).abs() <= 1e-2 * e.abs().max()).all())
        print(f"{m:5d}x{n:5d}x{k:5d}: off {statistics.median(ts[0]):8.1f} us {plans[0][:3]}   quarter "
              f"{statistics.median(ts[2]):8.1f} us {plans[2][:3]}   by cost {statistics.median(ts[1]):8.1f} us "
              f"{plans[1][:3]}  close {close}{same}", flush=True)


if __name__ == "__main__":
    main()
