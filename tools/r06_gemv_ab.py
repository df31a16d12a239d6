"""Lab A/B (lab build only) of k_gemv_4bit_bal variants on config 2 (11008 x 4096 nested, bf16): 14 rotating weight copies
replayed from one HIP graph (the bench leg), interleaved rounds; outputs compared bit for bit with the default."""
import ctypes as ct
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402

import python_src_quants.functional as F  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    res = {}
    for n_out, k_in in ((11008, 4096), (4096, 4096), (4096, 11008)):
        g = torch.Generator(device=dev).manual_seed(2)
        x = torch.randn(1, k_in, device=dev, dtype=torch.bfloat16, generator=g)
        out = torch.empty(1, n_out, device=dev, dtype=torch.bfloat16)
        ws = []
        for _ in range(14):
            W = (torch.randn(n_out, k_in, device=dev, generator=g) * 0.02).to(torch.bfloat16)
            ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
            del W
        arms = {"default": 0, "no_issue_barrier": 1, "weights_first": 2}
        times = {a: [] for a in arms}
        refs = {}
        for rnd in range(6):
            for a, bits in arms.items():
                F.lib.cgemv_4bit_lab_bits(ct.c_int(bits))
                calls = [(lambda q=q, st=st: F.gemv_4bit(x, q.t(), out=out, state=st)) for q, st in ws]
                for c in calls:
                    c()
                torch.cuda.synchronize()
                if rnd == 0:
                    refs[a] = F.gemv_4bit(x, ws[0][0].t(), state=ws[0][1]).clone()
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr):
                    for c in calls:
                        c()
                for _ in range(3):
                    gr.replay()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    gr.replay()
                e.record()
                torch.cuda.synchronize()
                times[a].append(s.elapsed_time(e) / 20 / len(calls) * 1e3)
        F.lib.cgemv_4bit_lab_bits(ct.c_int(0))
        key = f"{n_out}x{k_in}"
        res[key] = {a: round(statistics.median(v), 3) for a, v in times.items()}
        res[key]["bit_identical"] = {a: bool(torch.equal(refs[a], refs["default"])) for a in arms}
        print(json.dumps({key: res[key]}), flush=True)


if __name__ == "__main__":
    main()
