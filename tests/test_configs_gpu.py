"""The BASELINE.json configurations at their full sizes, on the routes the product takes for them.

* Metric shape (M=4096, N=4096, K=11008, NF4 bs=64, nested statistics): functional.gemm_4bit as routed (and the
  fused kernel forced), against the fp64 oracle ref.gemm_4bit_dequant_ref (the reference's M > 1 algorithm,
  ref:autograd/_functions.py:491-507) on 256 sampled rows x all columns.
* Config 4: the three distinct Llama-2-7B projection shapes (4096x4096, 11008x4096, 4096x11008) at 2048 tokens and
  at the config's own 65,536 tokens (batch 32 x seq 2048).
* Config 5: one 8-way column shard of each Llama-2-70B projection (q/o 8192x8192, k/v 1024x8192,
  gate/up 28672x8192, down 8192x28672, each N/8) at 2048 tokens, from a full-size quantised weight sliced by
  parallel.shard_quantized_4bit (packed bytes, uint8 codes and second-level scales sliced: every 70B shard starts
  on a second-level block) -- its statistics decode to the full weight's exactly.
* Config 2 (decode) is covered in test_matmul4bit_gpu.py; config 3 and the int8 metric shape in
  test_int8_gpu.py (exact int32 against a float64 GPU product, then mm_dequant bit-exact).
Tolerance: BASELINE.md §5 -- |d| <= 2e-2 * rms + 2e-2 * |ref| for bf16 outputs, mean |d| < 0.115."""
import numpy as np
import pytest
import torch

from oracle import ref

pytestmark = pytest.mark.gpu


def _F():
    import python_src_quants.functional as F
    return F


def _check_rows(Y, X, q, absmax, N, K, code, rows):
    exp = ref.gemm_4bit_dequant_ref(X[rows].float().cpu().numpy(), q.cpu().numpy(), absmax.cpu().numpy(), N, K, 64,
                                    code.cpu().numpy(), "bf16")
    got = Y[rows].float().cpu().numpy().astype(np.float64)
    rms = np.sqrt(np.mean(exp ** 2))
    err = np.abs(got - exp)
    assert np.all(err <= 2e-2 * rms + 2e-2 * np.abs(exp)), float(err.max())
    assert err.mean() < 0.115


def _sample_rows(M, dev, n=256, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randperm(M, generator=g)[:n].sort().values.to(dev)


def _quantized(N, K, dev, seed):
    F = _F()
    g = torch.Generator(device=dev).manual_seed(seed)
    W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    del W
    return q, st


@pytest.mark.parametrize("route", ["routed", "hgemm", "fused"])
def test_metric_shape(dev, route):
    """The metric shape as routed (deterministic rule: dequantise + the hand-written k_hgemm), with k_hgemm forced,
    and with the one-kernel fused NF4 GEMM forced."""
    F = _F()
    M, N, K = 4096, 4096, 11008
    q, st = _quantized(N, K, dev, 1000)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=torch.Generator(device=dev).manual_seed(1))
    if route == "routed":
        assert F.gemm_4bit_static_route(M, N, K) == "hgemm"
        Y = F.gemm_4bit(X, q, st)
    else:
        Y = F.gemm_4bit(X, q, st, _route=route)
    _check_rows(Y, X, q, F._absmax_fp32(st), N, K, st.code, _sample_rows(M, dev))


@pytest.mark.parametrize("n_out,k_in", [(4096, 4096), (11008, 4096), (4096, 11008)])
def test_llama2_7b_prefill_65536_tokens(dev, n_out, k_in):
    """Config 4 at its own size: batch 32 x seq 2048 = 65,536 activation rows through each distinct Llama-2-7B
    projection shape, on the route the product takes there (k_hgemm), 256 sampled rows against the fp64 oracle."""
    F = _F()
    M = 65536
    assert F.gemm_4bit_static_route(M, n_out, k_in) == "hgemm"
    q, st = _quantized(n_out, k_in, dev, 7 * n_out + k_in)
    X = torch.randn(M, k_in, device=dev, dtype=torch.bfloat16,
                    generator=torch.Generator(device=dev).manual_seed(n_out - k_in))
    Y = F.gemm_4bit(X, q, st)
    assert Y.shape == (M, n_out)
    _check_rows(Y, X, q, F._absmax_fp32(st), n_out, k_in, st.code, _sample_rows(M, dev, seed=n_out // 3))


@pytest.mark.parametrize("n_out,k_in", [(4096, 4096), (11008, 4096), (4096, 11008)])
def test_llama2_7b_projections(dev, n_out, k_in):
    F = _F()
    M = 2048
    q, st = _quantized(n_out, k_in, dev, n_out + k_in)
    X = torch.randn(M, k_in, device=dev, dtype=torch.bfloat16)
    Y = F.gemm_4bit(X, q, st)
    assert Y.shape == (M, n_out)
    _check_rows(Y, X, q, F._absmax_fp32(st), n_out, k_in, st.code, _sample_rows(M, dev, seed=n_out))


@pytest.mark.parametrize("name,n_out,k_in", [("q_o", 8192, 8192), ("k_v", 1024, 8192), ("gate_up", 28672, 8192),
                                             ("down", 8192, 28672)])
def test_llama2_70b_shard(dev, name, n_out, k_in):
    """Rank 3 of 8: its N/8 rows of the quantised full weight, via the product's shard function."""
    F = _F()
    from python_src_quants.parallel import shard_quantized_4bit
    world, rank, M = 8, 3, 2048
    q, st = _quantized(n_out, k_in, dev, n_out // 7 + k_in)
    qs, sts = shard_quantized_4bit(q, st, world, rank)
    n = n_out // world
    assert sts.shape == (n, k_in) and sts.nested
    X = torch.randn(M, k_in, device=dev, dtype=torch.bfloat16)
    Y = F.gemm_4bit(X, qs, sts)
    assert Y.shape == (M, n)
    # every 70B shard starts on a second-level block: its statistics decode to the full weight's exactly
    full = F._absmax_fp32(st)[rank * n * k_in // 64:(rank + 1) * n * k_in // 64]
    part = F._absmax_fp32(sts)
    assert torch.equal(part, full)
    _check_rows(Y, X, qs, part, n, k_in, sts.code, _sample_rows(M, dev, seed=n))
    # and the shard's packed bytes are the full weight's rows [rank*n, (rank+1)*n)
    assert torch.equal(qs.reshape(-1), q.reshape(-1)[rank * n * k_in // 2:(rank + 1) * n * k_in // 2])


def test_measured_route_4096_tokens_gate_up(dev, monkeypatch, tmp_path):
    """BNB_ROUTE_TUNING mode on the gate/up projection at 4096 tokens (11008 x 4096 weight): the first call times the
    four routes (k_hgemm, torch's library GEMM, the rocBLAS-searched one, the fused kernel) and caches one; every forced
    route and the routed call are within the oracle tolerance, the cache is stable, the plan file holds the choice and
    a process that imports it routes the same way, and a call under HIP-graph capture neither measures nor fails."""
    F = _F()
    monkeypatch.setattr(F, "GEMM_4BIT_ROUTE_TUNING", True)
    plan = tmp_path / "plan.json"
    monkeypatch.setenv("BNB_ROUTE_PLAN", str(plan))
    monkeypatch.setattr(F, "_ROUTES", {})
    monkeypatch.setattr(F, "_ROUTE_PLAN_LOADED", [True])
    M, N, K = 4096, 11008, 4096
    q, st = _quantized(N, K, dev, 77)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=torch.Generator(device=dev).manual_seed(7))
    rows = _sample_rows(M, dev, n=128, seed=3)
    am = F._absmax_fp32(st)
    for route in F.GEMM_4BIT_ROUTES:
        Y = F.gemm_4bit(X, q, st, _route=route)
        _check_rows(Y, X, q, am, N, K, st.code, rows)
    Y = F.gemm_4bit(X, q, st)
    first = F.gemm_4bit_measured_route(X, st)
    assert first in F.GEMM_4BIT_ROUTES
    _check_rows(Y, X, q, am, N, K, st.code, rows)
    F.gemm_4bit(X, q, st)
    assert F.gemm_4bit_measured_route(X, st) == first
    # the plan file: a fresh table (another process) imports the same choice
    import json
    table = json.loads(plan.read_text())
    assert [r[-1] for r in table["routes"]] == [first]
    monkeypatch.setattr(F, "_ROUTES", {})
    assert F.import_routes(table) == 1 and F.gemm_4bit_measured_route(X, st) == first
    # capture: an unmeasured shape takes the static rule without timing anything
    X2 = X[:3072].contiguous()
    out = torch.empty(3072, N, device=dev, dtype=torch.bfloat16)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        F.gemm_4bit(X2, q, st, out=out, _route="library")      # workspaces allocated outside the capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            F.gemm_4bit(X2, q, st, out=out)
    torch.cuda.current_stream().wait_stream(s)
    assert F.gemm_4bit_measured_route(X2, st) is None
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    _check_rows(out, X2, q, am, N, K, st.code, rows[rows < 3072])


_REPRO_SCRIPT = r"""
import hashlib, sys, torch
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/bitsandbytes-sycl_amd"]
import python_src_quants.functional as F
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1000)
W = (torch.randn(4096, 11008, device=dev, generator=g) * 0.02).to(torch.bfloat16)
q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
X = torch.randn(4096, 11008, device=dev, dtype=torch.bfloat16, generator=torch.Generator(device=dev).manual_seed(1))
Y = F.gemm_4bit(X, q, st)
torch.cuda.synchronize()
print("DIGEST", hashlib.sha256(Y.view(torch.int16).cpu().numpy().tobytes()).hexdigest())
"""


def test_metric_shape_bits_reproducible_across_processes(dev):
    """Two fresh processes (default, deterministic routing) compute the metric-shape product and return the same
    bits: the route does not depend on per-process timing."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("BNB_ROUTE_TUNING", "BNB_ROUTE_PLAN")}
    digests = []
    for _ in range(2):
        r = subprocess.run([sys.executable, "-c", _REPRO_SCRIPT, root], capture_output=True, text=True, env=env,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        digests.append([ln for ln in r.stdout.splitlines() if ln.startswith("DIGEST")][0])
    assert digests[0] == digests[1]


@pytest.mark.parametrize("nested", [False, True])
def test_fused_projections_70b_shard(dev, nested):
    """Config 5 decode with the projections that share an input fused (parallel.fuse_quantized_4bit): one rank's
    q/k/v (1024 + 128 + 128 rows) and gate/up (2 x 3584 rows) x 8192.  Packed bytes (and plain statistics)
    concatenate exactly; nested statistics are re-compressed for the fused weight and decode within the nested code's
    resolution of the parts'.  The fused GEMV and few-token GEMM agree with the fp64 oracle on the fused state, and
    each column range with the part's own GEMV within the GEMV tolerance."""
    F = _F()
    from python_src_quants.parallel import fuse_quantized_4bit, split_fused_columns
    torch.manual_seed(11 + nested)
    K = 8192
    for rows in ((1024, 128, 128), (3584, 3584)):
        parts = []
        for n in rows:
            W = (torch.randn(n, K, device=dev) * 0.02).to(torch.bfloat16)
            parts.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=nested))
            del W
        q, st, offs = fuse_quantized_4bit(parts)
        N = sum(rows)
        assert st.shape == (N, K) and offs == [0] + list(np.cumsum(rows))
        assert torch.equal(q.reshape(-1), torch.cat([p.reshape(-1) for p, _ in parts]))
        am_f = F._absmax_fp32(st)
        am_p = torch.cat([F._absmax_fp32(s) for _, s in parts])
        if nested:
            assert (am_f - am_p).abs().max().item() <= 0.02 * am_p.abs().max().item()
        else:
            assert torch.equal(am_f, am_p)
        for M in (1, 8):
            X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            Y = F.gemv_4bit(X, q.t(), state=st) if M == 1 else F.gemm_4bit(X, q, st)
            Y = Y.reshape(M, N)
            exp = ref.gemm_4bit_dequant_ref(X.float().cpu().numpy(), q.cpu().numpy(), am_f.cpu().numpy(), N, K, 64,
                                            st.code.cpu().numpy(), "bf16")
            rms = np.sqrt(np.mean(exp ** 2))
            err = np.abs(Y.float().cpu().numpy().astype(np.float64) - exp)
            assert np.all(err <= 2e-2 * rms + 2e-2 * np.abs(exp)), float(err.max())
            for (pq, pst), y in zip(parts, split_fused_columns(Y, offs)):
                yp = (F.gemv_4bit(X, pq.t(), state=pst) if M == 1 else F.gemm_4bit(X, pq, pst)).reshape(M, -1).float()
                r = yp.pow(2).mean().sqrt().item()
                assert (y.float() - yp).abs().max().item() <= 4e-2 * r + 4e-2 * yp.abs().max().item()


def test_hgemm_chunked_rows_beyond_4gib(dev):
    """a prompt whose activations exceed one k_hgemm launch's 32-bit offsets (rows * K * 2 > 4 GiB:
    524,588 rows x 4096) stays on the hand-written route -- row chunks of whole 256-row tiles, each multiplied straight
    into its rows of the output -- instead of the library GEMM; sampled rows on both sides of the chunk boundary
    against the fp64 oracle."""
    F = _F()
    M, N, K = 524288 + 300, 512, 4096
    assert M * K * 2 > 2 ** 32 and not F._hgemm_fits(M, N, K)
    assert F.gemm_4bit_static_route(M, N, K) == "hgemm"
    rc, nc = F._hgemm_chunks(M, N, K, 64)
    assert nc == N and rc % 256 == 0 and (rc - 1) * K * 2 + 2 * K <= 0xFFFFFFFF < M * K * 2
    q, st = _quantized(N, K, dev, 4242)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=torch.Generator(device=dev).manual_seed(5))
    Y = F.gemm_4bit(X, q, st)
    rows = torch.cat([_sample_rows(M, dev, n=120, seed=9),
                      torch.tensor([0, rc - 2, rc - 1, rc, rc + 1, M - 1], device=dev)]).unique()
    _check_rows(Y, X, q, F._absmax_fp32(st), N, K, st.code, rows)
    del X, Y
    torch.cuda.empty_cache()


def test_hgemm_chunked_weight_beyond_2g_elements(dev):
    """A weight of more than 2^31 elements (262,400 x 8192: its bf16 copy exceeds 4 GiB) on the hand-written route:
    dequantised one weight-row chunk at a time (whole statistics blocks), each chunk's product written into its
    columns of the output (ldc = N).  Random packed bytes and statistics (no float weight of that size is needed);
    sampled rows x sampled columns on both sides of the chunk boundary against the fp64 oracle on those columns."""
    F = _F()
    M, N, K = 2048, 262144 + 256, 8192
    assert N * K > 2 ** 31 and not F._hgemm_fits(M, N, K)
    assert F.gemm_4bit_static_route(M, N, K) == "hgemm"
    rc, nc = F._hgemm_chunks(M, N, K, 64)
    assert rc == M and nc % 256 == 0 and nc < N and nc * K < 2 ** 31
    g = torch.Generator(device=dev).manual_seed(77)
    q = torch.randint(0, 256, (N * K // 2, 1), device=dev, dtype=torch.uint8, generator=g)
    am = torch.rand(N * K // 64, device=dev, generator=g) * 0.05 + 0.01
    st = F.QuantState(absmax=am, shape=torch.Size([N, K]), code=F.get_4bit_type("nf4", device=dev), blocksize=64,
                      quant_type="nf4", dtype=torch.bfloat16)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
    Y = F.gemm_4bit(X, q, st)
    cols = torch.cat([torch.randperm(N, generator=torch.Generator().manual_seed(3))[:200].to(dev),
                      torch.tensor([0, nc - 1, nc, nc + 1, N - 1], device=dev)]).unique()
    rows = _sample_rows(M, dev, n=64, seed=4)
    qs = q.view(N, K // 2)[cols].contiguous()
    ams = am.view(N, K // 64)[cols].contiguous()
    exp = ref.gemm_4bit_dequant_ref(X[rows].float().cpu().numpy(), qs.cpu().numpy(), ams.cpu().numpy(), cols.numel(),
                                    K, 64, st.code.cpu().numpy(), "bf16")
    got = Y[rows][:, cols].float().cpu().numpy().astype(np.float64)
    rms = np.sqrt(np.mean(exp ** 2))
    err = np.abs(got - exp)
    assert np.all(err <= 2e-2 * rms + 2e-2 * np.abs(exp)), float(err.max())
    del X, Y, q
    torch.cuda.empty_cache()
