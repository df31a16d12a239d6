"""Time the few-token NF4 products (2..64 activation rows) of whichever library BNB_HIP_LIBRARY names (round 6 A/B of
variant builds; run once per library per round, rounds interleaved by the caller).  Per (weight, rows): 14 rotating
nested-NF4 weight copies replayed from one HIP graph (the bench's few-token leg), us per call, and a checksum of one
output so variants can be compared bit for bit.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402

import python_src_quants.functional as F  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    res = {"lib": os.path.basename(os.environ.get("BNB_HIP_LIBRARY", "product"))}
    for n_out, k_in in ((11008, 4096), (4096, 11008)):
        g = torch.Generator(device=dev).manual_seed(3)
        ws = []
        for _ in range(14):
            W = (torch.randn(n_out, k_in, device=dev, generator=g) * 0.02).to(torch.bfloat16)
            ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
            del W
        for m in (2, 8, 16, 32, 48, 64):
            x = torch.randn(m, k_in, device=dev, dtype=torch.bfloat16, generator=g)
            y = torch.empty(m, n_out, device=dev, dtype=torch.bfloat16)
            calls = [(lambda q=q, st=st: F.gemm_4bit(x, q, st, out=y)) for q, st in ws]
            for c in calls:
                c()
            torch.cuda.synchronize()
            ref = F.gemm_4bit(x, ws[0][0], ws[0][1])
            bits = ref.view(torch.int16).to(torch.int64).flatten()
            chk = int((bits * torch.arange(1, bits.numel() + 1, device=dev, dtype=torch.int64)).sum().item())
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for c in calls:
                    c()
            for _ in range(3):
                gr.replay()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    gr.replay()
                e.record()
                torch.cuda.synchronize()
                ts.append(s.elapsed_time(e) / 10 / len(calls) * 1e3)
            ts.sort()
            res[f"{n_out}x{k_in}@{m}"] = {"us": round(ts[2], 3), "checksum": chk}
        del ws
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
