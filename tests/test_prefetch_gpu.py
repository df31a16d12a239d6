"""The dequantise of the NEXT weight inside k_hgemm (chgemm_tn_pf_*, hgemm.hip HgSide; gemm_4bit(..., prefetch=...)).

Two things must hold bit for bit:
  * the GEMM's own output equals the plain k_hgemm launch (chgemm_tn_ws_*) -- the side work must not disturb it;
  * the weight it writes equals the dequantise kernel's (F.dequantize_4bit: k_dequantize_4bit_stream, itself pinned to
    the oracle by tests/test_quant_gpu.py) for NF4 / FP4, plain and nested statistics, bf16 / fp16,
on every launch plan (256 x 256, 256 x 128, 128 x 256 tiles; split-K) and with the side iterations in the main loop,
in the tail after it (few k-tiles, large next weight) and past the end of a tiny next weight.  Then the pipelined
gemm_4bit chain (each call prefetching the next weight) against the unpipelined calls."""
import pytest
import torch

pytestmark = pytest.mark.gpu

import python_src_quants.functional as F  # noqa: E402
from python_src_quants.cextension import lib  # noqa: E402


def _plan(m, n, k):
    import ctypes as ct
    out = (ct.c_int * 4)()
    lib.chgemm_tn_plan(ct.c_int(m), ct.c_int(n), ct.c_int(k), out)
    return tuple(out)


def _weight(n, k, dtype, qt, nested, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    W = (torch.randn(n, k, device="cuda", generator=g) * 0.02).to(dtype)
    return F.quantize_4bit(W, blocksize=64, quant_type=qt, compress_statistics=nested)


def _plain_gemm(X, W):
    import ctypes as ct
    rows, K = X.shape
    N = W.shape[0]
    out = torch.empty(rows, N, device="cuda", dtype=X.dtype)
    wsb = int(lib.chgemm_tn_workspace_bytes(ct.c_int32(rows), ct.c_int32(N), ct.c_int32(K)))
    ws = F._gemm_workspace(X.device, wsb)
    fn = lib.chgemm_tn_ws_bf16 if X.dtype == torch.bfloat16 else lib.chgemm_tn_ws_fp16
    F.post_call(F.pre_call(X.device))       # bind the library to torch's current stream (as gemm_4bit does)
    assert fn(ct.c_int32(rows), ct.c_int32(N), ct.c_int32(K), F.get_ptr(X), ct.c_int32(K), F.get_ptr(W), ct.c_int32(K),
              F.get_ptr(out), ct.c_int32(N), F.get_ptr(ws), ct.c_longlong(wsb)) == 0
    return out


def _pf_gemm(X, W, pf):
    import ctypes as ct
    rows, K = X.shape
    N = W.shape[0]
    out = torch.empty(rows, N, device="cuda", dtype=X.dtype)
    sn = pf[1]
    target = torch.full((sn.shape[0] * sn.shape[1],), float("nan"), device="cuda", dtype=X.dtype)
    wsb = int(lib.chgemm_tn_workspace_bytes(ct.c_int32(rows), ct.c_int32(N), ct.c_int32(K)))
    ws = F._gemm_workspace(X.device, wsb)
    F.post_call(F.pre_call(X.device))       # bind the library to torch's current stream (as gemm_4bit does)
    rc = F._launch_prefetch_gemm(X, W, out, ws, wsb, pf, target)
    assert rc == 0, rc
    return out, target.view(sn.shape[0], sn.shape[1])


# the two side-dequantise forms: 1 = the tail form (default since round 6: after the tile's epilogue, chunks taken by
# work stealing), 129 = the round-4 in-loop form (side steps between the MFMAs); both non-temporal side loads
FORMS = [1, 129]


@pytest.fixture(params=FORMS, ids=["tail", "inloop"])
def side_form(request):
    prev = lib.chgemm_set_side_mode(request.param)
    yield request.param
    lib.chgemm_set_side_mode(prev)


# (rows, N, K) of the GEMM -> its launch plan (WI, WJ, splits)
GEMMS = [
    ((4096, 4096, 2048), (8, 8, 1)),
    ((2048, 4096, 4096), (8, 4, 1)),
    ((96, 11008, 4096), (4, 8, 5)),
    ((4096, 1024, 8192), (8, 4, 2)),
]


@pytest.mark.parametrize("gemm,plan", GEMMS, ids=[f"{g[0]}x{g[1]}x{g[2]}" for g, _ in GEMMS])
@pytest.mark.parametrize("qt,nested", [("nf4", True), ("nf4", False), ("fp4", True), ("fp4", False)])
def test_prefetch_gemm_bits(gemm, plan, qt, nested, side_form):
    rows, N, K = gemm
    assert _plan(rows, N, K)[:3] == plan
    dtype = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(5)
    X = (torch.randn(rows, K, device="cuda", generator=g)).to(dtype)
    W = (torch.randn(N, K, device="cuda", generator=g) * 0.02).to(dtype)
    q2, s2 = _weight(11008, 4096, dtype, qt, nested, 7)
    out, nxt = _pf_gemm(X, W, (q2, s2))
    ref_out = _plain_gemm(X, W)
    ref_w = F.dequantize_4bit(q2, s2)
    torch.cuda.synchronize()
    assert torch.equal(out, ref_out)
    assert torch.equal(nxt, ref_w.view_as(nxt))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", ["tail", "tiny", "ragged"])
def test_prefetch_tail_and_edges(dtype, case, side_form):
    """tail: 2 k-tiles, so one side step in the loop and the rest after it; tiny: a 64 x 64 next weight (most
    workgroups own nothing); ragged: a next weight whose dwords do not fill the last workgroup's share."""
    rows, N, K = {"tail": (4096, 4096, 128), "tiny": (4096, 4096, 1024), "ragged": (2048, 4096, 4096)}[case]
    nn, kk = {"tail": (11008, 4096), "tiny": (64, 64), "ragged": (1003, 192)}[case]
    g = torch.Generator(device="cuda").manual_seed(11)
    X = (torch.randn(rows, K, device="cuda", generator=g)).to(dtype)
    W = (torch.randn(N, K, device="cuda", generator=g) * 0.02).to(dtype)
    for qt, nested in (("nf4", True), ("fp4", False)):
        q2, s2 = _weight(nn, kk, dtype, qt, nested, 13)
        out, nxt = _pf_gemm(X, W, (q2, s2))
        ref_out = _plain_gemm(X, W)
        ref_w = F.dequantize_4bit(q2, s2)
        torch.cuda.synchronize()
        assert torch.equal(out, ref_out), (case, qt)
        assert torch.equal(nxt, ref_w.view_as(nxt)), (case, qt)


def test_prefetch_declines_unsupported():
    """A next weight the side path does not take (element count % 32: each lane moves 32 weights) launches nothing and
    says so (1)."""
    dtype = torch.bfloat16
    X = torch.randn(256, 1024, device="cuda").to(dtype)
    W = torch.randn(1024, 1024, device="cuda").to(dtype)
    q2, s2 = _weight(8, 12, dtype, "nf4", False, 3)          # 96 elements: fine
    out, nxt = _pf_gemm(X, W, (q2, s2))
    torch.cuda.synchronize()
    assert torch.equal(nxt, F.dequantize_4bit(q2, s2).view_as(nxt))
    q3, s3 = _weight(3, 8, dtype, "nf4", False, 3)           # 24 elements: not a whole 32-weight group
    target = torch.empty(24, device="cuda", dtype=dtype)
    rc = F._launch_prefetch_gemm(X, W, torch.empty(256, 1024, device="cuda", dtype=dtype), None, 0, (q3, s3), target)
    assert rc == 1


@pytest.mark.parametrize("nested", [True, False])
def test_gemm_4bit_prefetch_chain_matches_unpipelined(nested):
    """A chain of gemm_4bit calls, each prefetching the next weight (three different weights, then the first again):
    every output equals the unpipelined call, and each prefetched weight is consumed by exactly the next call."""
    dtype = torch.bfloat16
    rows = 4096
    shapes = [(4096, 4096), (11008, 4096), (4096, 11008), (4096, 4096)]
    qs = [_weight(n, k, dtype, "nf4", nested, 20 + i) for i, (n, k) in enumerate(shapes[:3])]
    qs.append(qs[0])
    g = torch.Generator(device="cuda").manual_seed(1)
    xs = [torch.randn(rows, k, device="cuda", generator=g).to(dtype) for _, k in shapes]
    refs = [F.gemm_4bit(x, q, s, _route="hgemm") for x, (q, s) in zip(xs, qs)]
    key = (torch.device("cuda", torch.cuda.current_device()), dtype, F._stream_key(torch.device("cuda", torch.cuda.current_device())))
    F._PF_READY.pop(key, None)
    outs = []
    for i, (x, (q, s)) in enumerate(zip(xs, qs)):
        pf = qs[i + 1] if i + 1 < len(qs) else None
        outs.append(F.gemm_4bit(x, q, s, prefetch=pf))
        if pf is not None:
            assert F._PF_READY.get(key) is not None and F._PF_READY[key][1] == F._weight_meta(pf[0], pf[1], None)
        else:
            assert F._PF_READY.get(key) is None
    torch.cuda.synchronize()
    for i, (o, r) in enumerate(zip(outs, refs)):
        assert torch.equal(o, r), i


def test_gemm_4bit_prefetch_same_weight_each_step_and_graph():
    """The bench's pattern -- one weight, each step prefetching it for the next -- alternates the two slots, and
    replays from a HIP graph (two steps per graph, so each replay starts and ends on the same slot)."""
    dtype = torch.bfloat16
    q, s = _weight(4096, 4096, dtype, "nf4", True, 40)
    x = torch.randn(4096, 4096, device="cuda").to(dtype)
    ref = F.gemm_4bit(x, q, s, _route="hgemm")
    dev = torch.device("cuda", torch.cuda.current_device())
    key = (dev, dtype, F._stream_key(dev))
    F._PF_READY.pop(key, None)
    slots_seen = []
    for _ in range(4):
        o = F.gemm_4bit(x, q, s, prefetch=(q, s))
        slots_seen.append(F._PF_READY[key][0])
        assert torch.equal(o, ref)
    assert slots_seen == [0, 1, 0, 1]
    # graph capture on a side stream (the pool keys by stream: the capture stream's own slots)
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        F.gemm_4bit(x, q, s, prefetch=(q, s))             # prime the capture stream's slot
        torch.cuda.current_stream().synchronize()
        out = torch.empty(4096, 4096, device="cuda", dtype=dtype)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=st):
            F.gemm_4bit(x, q, s, out=out, prefetch=(q, s))
            F.gemm_4bit(x, q, s, out=out, prefetch=(q, s))
    torch.cuda.current_stream().wait_stream(st)
    for _ in range(3):
        out.zero_()
        gr.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, ref)


def test_prefetch_tail_form_repeated_launches_and_streams():
    """The tail form over a next weight of many chunks per wave (11008 x 4096: 2,752 chunks of 1,024 dwords on 1,024
    waves), back to back on one stream and on a second stream, a NaN-filled target each time; plus the 128 x 128 tile
    with split-K, which only the tail form runs."""
    prev = lib.chgemm_set_side_mode(1)
    try:
        dtype = torch.bfloat16
        g = torch.Generator(device="cuda").manual_seed(17)
        q2, s2 = _weight(11008, 4096, dtype, "nf4", True, 19)
        ref_w = F.dequantize_4bit(q2, s2)
        for rows, N, K in ((4096, 4096, 1024), (512, 4096, 4096)):
            X = torch.randn(rows, K, device="cuda", generator=g).to(dtype)
            W = (torch.randn(N, K, device="cuda", generator=g) * 0.02).to(dtype)
            ref_out = _plain_gemm(X, W)
            for st in (torch.cuda.current_stream(), torch.cuda.Stream(), torch.cuda.current_stream()):
                st.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(st):
                    for _ in range(3):
                        out, nxt = _pf_gemm(X, W, (q2, s2))
                        st.synchronize()
                        assert torch.equal(out, ref_out), (rows, N, K)
                        assert torch.equal(nxt, ref_w.view_as(nxt)), (rows, N, K)
                torch.cuda.current_stream().wait_stream(st)
        assert _plan(512, 4096, 4096)[:2] == (4, 4)         # (the quarter tile took that one)
    finally:
        lib.chgemm_set_side_mode(prev)
