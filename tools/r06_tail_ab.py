"""A/B (round 6): the metric step and the C4 prefill layer with the next weight's dequantise
  pair   -- its own k_dequantize_4bit_stream launch before each k_hgemm (the bench default so far),
  tail   -- inside the previous k_hgemm, after each workgroup's tile, chunks taken by work stealing (chgemm_set_side_mode(1)),
  inloop -- inside the previous k_hgemm, between its MFMAs (the round-4 form, chgemm_set_side_mode(129)),
interleaved rounds in one process (same clock history for every arm), outputs compared bit for bit."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import python_src_quants.functional as F  # noqa: E402

M, N, K = 4096, 4096, 11008


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
    W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    del W
    Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    arms = {"pair": (None, 1), "tail": ((q, st), 1), "inloop": ((q, st), 129)}
    ref = F.gemm_4bit(X, q, st, out=torch.empty_like(Y)).clone()

    def run(arm, steps):
        pf, mode = arms[arm]
        F.lib.chgemm_set_side_mode(mode)
        for _ in range(3):
            F.gemm_4bit(X, q, st, out=Y, prefetch=pf)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(steps):
            F.gemm_4bit(X, q, st, out=Y, prefetch=pf)
        e.record()
        torch.cuda.synchronize()
        same = torch.equal(Y, ref)
        return s.elapsed_time(e) / steps * 1e3, same

    t_end = time.perf_counter() + 0.5          # clock ramp
    while time.perf_counter() < t_end:
        run("pair", 8)
    res = {a: [] for a in arms}
    same = {a: True for a in arms}
    for _ in range(7):
        for a in arms:
            us, ok = run(a, 40)
            res[a].append(us)
            same[a] &= ok
    out = {"metric_step_us": {a: {"median": statistics.median(v), "min": min(v), "all": [round(x, 1) for x in v]}
                              for a, v in res.items()},
           "bit_identical_to_pair": same}
    print(json.dumps(out), flush=True)
    # the C4 prefill layer (seven projections, 65,536 tokens) with each projection's GEMM dequantising the next one's weight
    c4 = {}
    for _ in range(2):
        for a, (pf, mode) in arms.items():
            F.lib.chgemm_set_side_mode(mode)
            bench.PREFETCH[0] = pf is not None
            c4.setdefault(a, []).append(bench.bench_llama2_7b_prefill(dev, iters=2)["layer_ms"])
    F.lib.chgemm_set_side_mode(1)
    bench.PREFETCH[0] = False
    print(json.dumps({"c4_layer_ms": {a: {"min": min(v), "all": [round(x, 3) for x in v]} for a, v in c4.items()}}),
          flush=True)


if __name__ == "__main__":
    main()
