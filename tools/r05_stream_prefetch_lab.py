"""Lab (GPU, round 5): the metric step's dequantise on a second stream, one weight ahead (the next step's weight
dequantised into the other of two slots while this step's k_hgemm runs), against the sequential pair on one stream.
k_hgemm holds every CU with one workgroup (256 tiles of 256 x 256, 512 registers per wave), so the dequantise's
workgroups only get CUs as GEMM workgroups finish: the overlap is the GEMM's tail (XCD spread + epilogue,
profiles/lab/r05_hgemm_timeline.txt).  Same weight every step, as in bench.py.  Prints us per step (median of rounds).
Usage: python tools/r05_stream_prefetch_lab.py [rounds]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    m, n, k = 4096, 4096, 11008
    Wf = (torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(Wf, blocksize=64, quant_type="nf4", compress_statistics=True)
    del Wf
    X = torch.randn(m, k, device=dev, dtype=torch.bfloat16, generator=g)
    Y = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    slots = [torch.empty(n, k, device=dev, dtype=torch.bfloat16) for _ in range(2)]
    ws_bytes = int(F.lib.chgemm_tn_workspace_bytes(m, n, k))
    ws = torch.empty(max(ws_bytes, 16) // 4 + 1, dtype=torch.float32, device=dev)
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    print(f"stream priorities: low {lo} high {hi}", flush=True)
    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    main_hi = torch.cuda.Stream(priority=hi)
    side_lo = torch.cuda.Stream(priority=lo)

    def gemm(W):
        F.pre_call(dev)
        assert F.lib.chgemm_tn_ws_bf16(m, n, k, F.get_ptr(X), k, F.get_ptr(W), k, F.get_ptr(Y), n, F.get_ptr(ws),
                                       ws_bytes) == 0

    def deq(W):
        assert F._dequant_4bit_nested(q, st, W)

    def sequential(steps):
        for _ in range(steps):
            deq(slots[0])
            gemm(slots[0])

    ev_deq = [torch.cuda.Event(), torch.cuda.Event()]
    ev_free = [torch.cuda.Event(), torch.cuda.Event()]

    def pipelined(steps, main_s=main_s, side=side):
        # step i's weight is in slot i % 2; step 0's dequantised on the main stream, step i + 1's on the side stream
        # after step i's GEMM launch, once the GEMM that last read that slot (step i - 1) is done
        deq(slots[0])
        for i in range(steps):
            cur, nxt = i % 2, (i + 1) % 2
            if i > 0:
                main_s.wait_event(ev_deq[cur])
            ev_free[nxt].record(main_s)          # everything before this GEMM, incl. step i - 1's GEMM on slot nxt
            gemm(slots[cur])
            if i + 1 < steps:
                side.wait_event(ev_free[nxt])
                with torch.cuda.stream(side):
                    deq(slots[nxt])
                    ev_deq[nxt].record(side)
        main_s.wait_stream(side)

    def timed(fn, steps=20):
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn(steps)
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / steps * 1e3

    sequential(3)
    ref = Y.clone()
    pipelined(3)
    torch.cuda.synchronize()
    print(f"pipelined == sequential bitwise: {torch.equal(Y, ref)}", flush=True)
    def pipelined_prio(steps):
        # the GEMMs on a high-priority stream, the dequantises on a low-priority one: when both become ready at once
        # (step i's dequantise done -> step i's GEMM and step i + 1's dequantise), the GEMM's workgroups dispatch first
        main_hi.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(main_hi):
            pipelined(steps, main_s=main_hi, side=side_lo)
        torch.cuda.current_stream().wait_stream(main_hi)

    Y.zero_()
    pipelined_prio(3)
    torch.cuda.synchronize()
    print(f"pipelined (priorities) == sequential bitwise: {torch.equal(Y, ref)}", flush=True)
    ts = {"sequential": [], "pipelined": [], "pipelined prio": []}
    for _ in range(rounds):
        ts["sequential"].append(timed(sequential))
        ts["pipelined"].append(timed(pipelined))
        ts["pipelined prio"].append(timed(pipelined_prio))
    for name, v in ts.items():
        print(f"{name:10s}: {statistics.median(v):7.1f} us per step  (min {min(v):7.1f}, max {max(v):7.1f})", flush=True)


if __name__ == "__main__":
    main()
