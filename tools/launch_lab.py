"""Lab (GPU): wave-entry ramp and streaming-landing ramp of a one-shot grid (tools/launch_lab.hip).
Each configuration launches `blocks` workgroups of `waves` waves with `lds` bytes of dynamic LDS; every wave streams
`per_wave` x 1 KiB (16 B per lane) from a contiguous chunk of a rotating set of 22.5 MB buffers (mid-stream, cold L2).
Prints entry / first-batch landed / done percentiles in us after the earliest entry.
Usage: python tools/launch_lab.py   (needs tools/_launch_lab.so, built by the hipcc line in launch_lab.hip)"""
import ctypes
import os
import sys

import numpy as np
import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_launch_lab.so"))
dev = torch.device("cuda", 0)
TOTAL = 11008 * 4096 // 2                      # the 11008 x 4096 NF4 weight, bytes
bufs = [torch.randint(0, 255, (TOTAL * 5 // 4,), dtype=torch.uint8, device=dev) for _ in range(14)]
sink = torch.zeros(16, dtype=torch.uint8, device=dev)


def run(blocks, waves, lds, per_wave):
    nw = blocks * waves
    st = torch.zeros(nw * 4, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    for it in range(3):
        for i, b in enumerate(bufs):
            rec = it == 2 and i == 7
            rc = lib.launch_lab(ctypes.c_void_p(b.data_ptr()), per_wave,
                                ctypes.c_void_p(st.data_ptr()),
                                ctypes.c_void_p(sink.data_ptr()), blocks, waves, lds, ctypes.c_void_p(stream))
            assert rc == 0, rc
            if rec:
                torch.cuda.synchronize()
                t = st.view(nw, 4).cpu().numpy().astype(np.int64).copy()
    torch.cuda.synchronize()
    t0 = t[:, 0].min()
    ent = (t[:, 0] - t0) / 100.0
    intra = ent.reshape(blocks, waves)
    intra = intra.max(axis=1) - intra.min(axis=1)
    wg0 = ent.reshape(blocks, waves).min(axis=1)
    line = (f"blocks {blocks:4d} waves {waves} lds {lds // 1024:3d}K per_wave {per_wave:3d} ({nw * per_wave * 1024 / 1e6:5.1f} MB): "
            f"entry p50/p95/max {np.percentile(ent, 50):5.2f} {np.percentile(ent, 95):5.2f} {ent.max():5.2f}; "
            f"wg first-entry max {wg0.max():5.2f}; intra-wg spread p50/max {np.percentile(intra, 50):5.2f} {intra.max():5.2f}")
    if per_wave > 0:
        land = (t[:, 1] - t0) / 100.0
        done = (t[:, 2] - t0) / 100.0
        line += (f"; issued p50/max {np.percentile(land, 50):5.2f} {land.max():5.2f}; "
                 f"done p50/p95/max {np.percentile(done, 50):5.2f} {np.percentile(done, 95):5.2f} {done.max():5.2f}")
    print(line, flush=True)
    return t




def run_stream(mode, graph_us=True):
    rows = 11008
    nw = (rows + 47) // 48 * 8
    st = torch.zeros(nw * 4, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    for it in range(3):
        for i, b in enumerate(bufs):
            assert lib.stream_lab(ctypes.c_void_p(b.data_ptr()), rows, ctypes.c_void_p(st.data_ptr()),
                                  ctypes.c_void_p(sink.data_ptr()), mode, ctypes.c_void_p(stream)) == 0
            if it == 2 and i == 7:
                torch.cuda.synchronize()
                t = st.view(nw, 4).cpu().numpy().astype(np.int64).copy()
    # event timing over 14 rotating launches x 5
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for it in range(5):
        for b in bufs:
            lib.stream_lab(ctypes.c_void_p(b.data_ptr()), rows, ctypes.c_void_p(st.data_ptr()),
                           ctypes.c_void_p(sink.data_ptr()), mode, ctypes.c_void_p(stream))
    e1.record()
    torch.cuda.synchronize()
    per = e0.elapsed_time(e1) * 1000 / 70
    t0 = t[:, 0].min()
    ent, iss, done = [(t[:, i] - t0) / 100.0 for i in range(3)]
    names = {0: "plain nt contiguous", 1: "DMA nt contiguous", 2: "plain nt pattern", 3: "DMA nt pattern",
             4: "plain contiguous", 5: "DMA contiguous", 6: "plain pattern", 7: "DMA pattern",
             9: "DMA nt contig+tok", 10: "plain nt pattern+tok", 11: "DMA nt pattern+tok",
             16: "plain nt 16x64", 24: "plain nt 16x64+tok", 17: "DMA nt 16x64"}
    print(f"stream mode {mode} ({names[mode]:20s}): entry max {ent.max():5.2f}; issued p50/max {np.percentile(iss, 50):5.2f} "
          f"{iss.max():5.2f}; done p50/p95/max {np.percentile(done, 50):5.2f} {np.percentile(done, 95):5.2f} "
          f"{done.max():5.2f}; back-to-back launch {per:6.2f} us", flush=True)


for mode in (int(a) for a in os.environ.get("LAB_MODES", "0,1,2,3,4,5,6,7").split(",")):
    run_stream(mode)
if os.environ.get("LAB_RAMP", "1") == "0":
    sys.exit(0)

for per_wave in (0, None):
    for blocks, waves, lds in ((230, 8, 160 * 1024), (230, 8, 0), (256, 8, 96 * 1024), (460, 4, 112 * 1024),
                               (256, 4, 0), (512, 4, 80 * 1024), (1024, 2, 0), (256, 1, 0)):
        pw = 0 if per_wave == 0 else max(4, round(TOTAL / (blocks * waves * 1024) / 4) * 4)
        run(blocks, waves, lds, pw)
t = run(230, 8, 160 * 1024, 0)
hw = t[:, 3]
se = (hw >> 13) & 7
cu = (hw >> 8) & 15
simd = (hw >> 4) & 3
print("first 24 entries (us, se, cu, simd):",
      [(round((t[i, 0] - t[:, 0].min()) / 100.0, 2), int(se[i]), int(cu[i]), int(simd[i]))
       for i in np.argsort(t[:, 0])[:24]])
