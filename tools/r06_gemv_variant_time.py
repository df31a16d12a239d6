"""Time the decode GEMV of whichever library BNB_HIP_LIBRARY names (round 6 A/B of the variant builds of
tools/r06_gemv_variants.sh; run once per library per round, rounds interleaved by the caller).  Per shape: 14 rotating
nested-NF4 weight copies replayed from one HIP graph (the bench leg), us per call; plus a checksum of one output so the
variants can be compared bit for bit.  Prints one JSON line."""
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
    shapes = ((11008, 4096, True), (11008, 4096, False), (4096, 4096, True), (4096, 11008, True),
              (1280, 8192, True), (7168, 8192, True), (1024, 28672, True), (128, 8192, True))   # + the 70B rank shards
    for n_out, k_in, nested in shapes:
        g = torch.Generator(device=dev).manual_seed(2)
        x = torch.randn(1, k_in, device=dev, dtype=torch.bfloat16, generator=g)
        out = torch.empty(1, n_out, device=dev, dtype=torch.bfloat16)
        ws = []
        for _ in range(14):
            W = (torch.randn(n_out, k_in, device=dev, generator=g) * 0.02).to(torch.bfloat16)
            ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=nested))
            del W
        calls = [(lambda q=q, st=st: F.gemv_4bit(x, q.t(), out=out, state=st)) for q, st in ws]
        for c in calls:
            c()
        torch.cuda.synchronize()
        ref = F.gemv_4bit(x, ws[0][0].t(), state=ws[0][1])
        bits = ref.view(torch.int16).to(torch.int64)
        pos = torch.arange(1, bits.numel() + 1, device=dev, dtype=torch.int64)
        chk = int((bits.flatten() * pos).sum().item())
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for c in calls:
                c()
        for _ in range(5):
            gr.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                gr.replay()
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) / 20 / len(calls) * 1e3)
        ts.sort()
        res[f"{n_out}x{k_in}{'_nested' if nested else ''}"] = {"us": round(ts[2], 3), "checksum": chk}
        del ws
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
