"""Per-wave timeline of the decode GEMV k_gemv_4bit_bal, lab build only:
BNB_HIP_LIBRARY=<lab .so> [GV_LAB_BITS=<cgemv_4bit_lab_bits>] python tools/r06_gemv_timeline.py

Config 2 (Linear4bit NF4 11008 x 4096, nested statistics, bf16), 14 rotating weight copies launched back to back (the
bench leg's setting: > the 256 MB MALL, so the weights come from HBM); the stamps of the LAST launch are read (every
launch overwrites them).  Per wave, relative to the earliest wave start of that launch: start, statistics / activation
loads issued, weight loads issued, statistics + activations landed and table built, dots done, row stored.  Reports
p5 / p50 / p95 over the waves, and the same per XCD."""
import ctypes as ct
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import python_src_quants.functional as F  # noqa: E402

NAMES = ["start", "stats_acts_issued", "weights_issued", "stats_acts_landed_table_built", "dots_done", "row_stored"]


def main():
    dev = torch.device("cuda", 0)
    n_out, k_in, copies = 11008, 4096, 14
    g = torch.Generator(device=dev).manual_seed(2)
    x = torch.randn(1, k_in, device=dev, dtype=torch.bfloat16, generator=g)
    out = torch.empty(1, n_out, device=dev, dtype=torch.bfloat16)
    ws = []
    for _ in range(copies):
        W = (torch.randn(n_out, k_in, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
        del W
    buf = torch.zeros(4096 * 16 * 8, dtype=torch.int64, device=dev)
    assert F.lib.cgemv_4bit_lab_bits(ct.c_int(int(os.environ.get("GV_LAB_BITS", "0")))) == 0
    for q, st in ws:                                        # warm: code objects, plans
        F.gemv_4bit(x, q.t(), out=out, state=st)
    torch.cuda.synchronize()
    res = {}
    for rep in range(3):
        assert F.lib.cgemv_4bit_timeline(ct.c_void_p(buf.data_ptr())) == 0
        buf.zero_()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for q, st in ws:
            F.gemv_4bit(x, q.t(), out=out, state=st)
        e.record()
        torch.cuda.synchronize()
        F.lib.cgemv_4bit_timeline(ct.c_void_p(0))
        per_call_us = s.elapsed_time(e) / copies * 1e3
        t = buf.view(-1, 8).cpu().numpy()
        t = t[t[:, 0] != 0]
        t0 = t[:, 0].min()
        rel = (t[:, :6] - t0) * 0.01                       # 10 ns ticks -> us
        row = {"per_call_us_back_to_back": round(per_call_us, 3), "waves": int(len(t)),
               "launch_span_us": round(float(rel[:, 5].max()), 3)}
        for i, nm in enumerate(NAMES):
            row[nm] = [round(float(np.percentile(rel[:, i], p)), 3) for p in (5, 50, 95)]
        xcd = {}
        for xc in sorted(set(t[:, 6].tolist())):
            m = t[:, 6] == xc
            xcd[int(xc)] = {"dots_done_p50": round(float(np.percentile(rel[m, 4], 50)), 3),
                            "row_stored_max": round(float(rel[m, 5].max()), 3)}
        row["by_xcd"] = xcd
        res[f"rep{rep}"] = row
        print(json.dumps({f"rep{rep}": row}), flush=True)


if __name__ == "__main__":
    main()
