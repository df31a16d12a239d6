"""Lab (GPU): per-wave timeline of the 256 x 256 k_hgemm (HG_V_TL variant, chgemm_timeline): where the fixed cost of a
launch goes.  Stamps (s_memrealtime, 10 ns): start, prologue done (tile 0 landed), k-loop done, epilogue stores issued,
stores complete.  Shapes: bf16 4096 x 4096 x 11008 (the metric GEMM: 256 tiles, one per CU) alone and inside the
metric step (after the dequantise), bf16 4096^3.  Prints percentiles over waves, in us after the earliest start.
Usage: python tools/hgemm_timeline.py"""
import ctypes as ct
import os
import sys
os.environ.setdefault("BNB_HIP_LIBRARY", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                   "bitsandbytes-sycl_amd", "build", "libbitsandbytes_hip_lab.so"))   # lab hooks: `make -C bitsandbytes-sycl_amd/csrc lab`

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402


def report(name, buf, nwg):
    t = buf[: nwg * 4 * 8].view(nwg * 4, 8).cpu().numpy().astype(np.int64)
    t0 = t[:, 0].min()
    rel = (t[:, :5] - t0) / 100.0
    names = ["start", "prologue done", "loop done", "stores issued", "stores landed"]
    print(f"== {name}: {nwg} workgroups", flush=True)
    for i, nm in enumerate(names):
        p = np.percentile(rel[:, i], [0, 5, 50, 95, 100])
        print(f"   {nm:15s} min {p[0]:7.2f}  p5 {p[1]:7.2f}  p50 {p[2]:7.2f}  p95 {p[3]:7.2f}  max {p[4]:7.2f}", flush=True)
    d = np.diff(rel, axis=1)
    for i, nm in enumerate(["prologue", "loop", "epilogue issue", "store drain"]):
        p = np.percentile(d[:, i], [5, 50, 95])
        print(f"   {nm:15s} dur p5 {p[0]:7.2f}  p50 {p[1]:7.2f}  p95 {p[2]:7.2f}", flush=True)
    # by dispatch group (blockIdx % 8: the blocks that share an XCD) and by physical XCD (HW_REG_XCC_ID): if the slow
    # group moves with the physical XCD across launches it is the hardware, if it stays with blockIdx % 8 the data
    grp = (np.arange(nwg * 4) // 4) % 8
    xcc = t[:, 6]
    print("   loop done p50 by blockIdx % 8: " + " ".join(f"{np.median(rel[grp == x, 2]):.2f}" for x in range(8)), flush=True)
    print("   loop done p50 by XCC_ID:       " + " ".join(f"{np.median(rel[xcc == x, 2]):.2f}" if (xcc == x).any() else "  -  "
                                                    for x in range(8)), flush=True)
    print("   XCC_ID of blockIdx 0..7: " + " ".join(str(int(xcc[4 * b])) for b in range(8)), flush=True)


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    buf = torch.zeros(4096 * 4 * 8, dtype=torch.int64, device=dev)
    for (m, n, k) in [(4096, 4096, 11008), (4096, 4096, 4096)]:
        X = torch.randn(m, k, device=dev, dtype=torch.bfloat16, generator=g)
        W = (torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        Y = torch.empty(m, n, device=dev, dtype=torch.bfloat16)

        def run():
            F.pre_call(dev)
            assert F.lib.chgemm_tn_bf16(m, n, k, F.get_ptr(X), k, F.get_ptr(W), k, F.get_ptr(Y), n) == 0
        for _ in range(5):
            run()
        ref = Y.clone()
        assert F.lib.chgemm_timeline(ct.c_void_p(buf.data_ptr())) == 0
        for rep in range(3):
            run()
            torch.cuda.synchronize()
            report(f"bf16 k_hgemm {m}x{n}x{k} (launch {rep})", buf, 256)
        assert F.lib.chgemm_timeline(None) == 0
        assert torch.equal(Y, ref)                       # the timeline variant computes the same bits
    # the same GEMM with each XCD on the other half of the N-tiles (a bijection of the tile map: same outputs): does the
    # slow group follow the XCD or the data?
    m, n, k = 4096, 4096, 11008
    X = torch.randn(m, k, device=dev, dtype=torch.bfloat16, generator=g)
    W = (torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    Y = torch.empty(m, n, device=dev, dtype=torch.bfloat16)

    def run2():
        F.pre_call(dev)
        assert F.lib.chgemm_tn_bf16(m, n, k, F.get_ptr(X), k, F.get_ptr(W), k, F.get_ptr(Y), n) == 0
    for _ in range(3):
        run2()
    ref = Y.clone()
    assert F.lib.chgemm_timeline(ct.c_void_p(buf.data_ptr())) == 0
    for swap in (0, 1, 0, 1):
        assert F.lib.chgemm_timeline_nswap(swap) == 0
        run2()
        torch.cuda.synchronize()
        assert torch.equal(Y, ref)
        report(f"bf16 k_hgemm {m}x{n}x{k}, N halves swapped between XCD pairs: {swap}", buf, 256)
    assert F.lib.chgemm_timeline_nswap(0) == 0
    # ablation: the epilogue with its C stores dropped (issued against a zero-record buffer): conversion + staging +
    # store issue without the memory write -- what the 32 MB write itself costs
    for nostore in (1, 0):
        assert F.lib.chgemm_timeline_nostore(nostore) == 0
        run2()
        torch.cuda.synchronize()
        report(f"bf16 k_hgemm {m}x{n}x{k}, C stores dropped: {nostore}", buf, 256)
    assert F.lib.chgemm_timeline_nostore(0) == 0
    run2()
    torch.cuda.synchronize()
    assert torch.equal(Y, ref)
    assert F.lib.chgemm_timeline(None) == 0
    # the metric step: dequantise + k_hgemm, the GEMM stamped
    m, n, k = 4096, 4096, 11008
    Wq = (torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(Wq, blocksize=64, quant_type="nf4", compress_statistics=True)
    X = torch.randn(m, k, device=dev, dtype=torch.bfloat16, generator=g)
    Y = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    for _ in range(5):
        F.gemm_4bit(X, q, st, out=Y)
    assert F.lib.chgemm_timeline(ct.c_void_p(buf.data_ptr())) == 0
    for _ in range(3):
        F.gemm_4bit(X, q, st, out=Y)
    torch.cuda.synchronize()
    assert F.lib.chgemm_timeline(None) == 0
    report("metric step's k_hgemm (after the dequantise)", buf, 256)


if __name__ == "__main__":
    main()
