"""Round 5 A/B: the metric step's dequantise launch shape (cdequantize_set_stream_cfg: packed dwords per lane per pass
p = 4 / 8 / 16, grid cap 0 / 1024 / 2048 / 4096) inside the step (gemm_4bit = dequantise + k_hgemm at 4096 x 4096 x
11008, NF4 nested) and alone back to back; medians of interleaved rounds; outputs bit-identical.
Usage: python tools/r05_dq_cfg_ab.py [rounds]"""
import os
import statistics
import sys

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
    W = (torch.randn(4096, 11008, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    del W
    X = torch.randn(4096, 11008, device=dev, dtype=torch.bfloat16, generator=g)
    Y = torch.empty(4096, 4096, device=dev, dtype=torch.bfloat16)
    Wd = torch.empty(4096, 11008, device=dev, dtype=torch.bfloat16)
    cfgs = [(8, 0), (4, 0), (16, 0), (8, 1024), (8, 2048), (8, 4096), (16, 2048), (4, 4096)]
    step = lambda: F.gemm_4bit(X, q, st, out=Y)  # noqa: E731
    deq = lambda: F._dequant_4bit_nested(q, st, Wd)  # noqa: E731
    ref = None
    for p, cap in cfgs:
        F.lib.cdequantize_set_stream_cfg(p, cap)
        deq()
        torch.cuda.synchronize()
        if ref is None:
            ref = Wd.clone()
        assert torch.equal(Wd, ref), (p, cap)
    ts = {c: [] for c in cfgs}
    td = {c: [] for c in cfgs}
    for _ in range(rounds):
        for c in cfgs:
            F.lib.cdequantize_set_stream_cfg(*c)
            for _ in range(3):
                step()
            ts[c].append(timed(step))
            td[c].append(timed(deq))
    F.lib.cdequantize_set_stream_cfg(8, 0)
    for c in cfgs:
        print(f"p {c[0]:2d} grid cap {c[1]:5d}: metric step {statistics.median(ts[c]):7.1f} us   dequantise alone "
              f"{statistics.median(td[c]):6.2f} us", flush=True)


if __name__ == "__main__":
    main()
