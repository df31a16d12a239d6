"""Seeded random-shape parity sweep (round 5): shapes drawn across every route of the two product entry points, each
checked against the oracle -- beyond the hand-picked grids of the other files.

* gemm_4bit (the M>1 slot of cgemm_4bit_inference, ref:pythonInterface.cpp:377; dequantize_4bit + F.linear,
  ref:autograd/_functions.py:491-507): activation rows 1..2500 (the GEMV, multi-row GEMV, few-token, 33..64-token,
  fused and dequantise + k_hgemm routes), out-features 16..6000 (ragged), in-features multiples of 64 up to 8192,
  NF4 / FP4, blocksize 64 / 128 / 256, plain / nested statistics, bf16 / fp16.  Bar: the GEMV / tile-kernel
  tolerance of tests/test_t64_gpu.py against the fp64 oracle of the dequantised weight (at most 48 sampled rows);
  deterministic over two calls.
* igemmlt + fused mm_dequant (ref:op_gemm.cpp:541-655, kernel_quant.cpp:3969): random int8 shapes, the int32 product
  exact and the fp16 outputs bit for bit against the oracle's mm_dequant order.
The draws are fixed by the seed, so a failure names a reproducible case."""
import numpy as np
import pytest
import torch

from oracle import ref

pytestmark = pytest.mark.gpu

_ROWS = [1, 2, 3, 4, 5, 8, 13, 16, 17, 31, 32, 33, 40, 47, 48, 57, 63, 64, 65, 96, 128, 200, 256, 300, 513, 1024,
         2048, 2500]


def _gemm_cases(n_cases=96, seed=20265):
    rng = np.random.default_rng(seed)
    cases = []
    for i in range(n_cases):
        M = int(rng.choice(_ROWS))
        N = int(rng.integers(16, 6001))
        K = 64 * int(rng.integers(1, 129))
        if M >= 1024:                                 # keep the oracle's dequantised weight small at large M
            K = min(K, 2048)
            N = min(N, 3000)
        bs = int(rng.choice([64, 64, 128, 256]))
        if K % bs:
            bs = 64
        cases.append((i, M, N, K, bs, str(rng.choice(["nf4", "fp4"])), bool(rng.integers(0, 2)),
                      str(rng.choice(["bf16", "fp16"]))))
    return cases


@pytest.mark.parametrize("case", _gemm_cases(), ids=lambda c: f"c{c[0]}-M{c[1]}-N{c[2]}-K{c[3]}-bs{c[4]}-{c[5]}"
                                                            f"-{'n' if c[6] else 'p'}-{c[7]}")
def test_gemm_4bit_random_shapes_vs_oracle(dev, case):
    import python_src_quants.functional as F
    i, M, N, K, bs, qt, nested, dt = case
    dtype = torch.bfloat16 if dt == "bf16" else torch.float16
    g = torch.Generator(device=dev).manual_seed(1000 + i)
    W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(dtype)
    X = torch.randn(M, K, device=dev, dtype=dtype, generator=g)
    q, st = F.quantize_4bit(W, blocksize=bs, quant_type=qt, compress_statistics=nested)
    del W
    Y = F.gemm_4bit(X, q, st)
    Y2 = F.gemm_4bit(X, q, st)
    assert Y.shape == (M, N) and Y.dtype == dtype
    assert torch.equal(Y, Y2)
    rows = np.sort(np.random.default_rng(i).choice(M, size=min(M, 48), replace=False))
    absmax = F._absmax_fp32(st).cpu().numpy()
    exp = ref.gemm_4bit_dequant_ref(X[torch.from_numpy(rows).to(dev)].float().cpu().numpy(), q.cpu().numpy(), absmax,
                                    N, K, bs, st.code.cpu().numpy(), dt)
    got = Y[torch.from_numpy(rows).to(dev)].float().cpu().numpy()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-2
    rms = float(np.sqrt(np.mean(exp ** 2))) + 1e-12
    bad = np.abs(got - exp) > tol * rms + tol * np.abs(exp)
    assert not bad.any(), (float(bad.mean()), float(np.max(np.abs(got - exp))), F.gemm_4bit_static_route(M, N, K))


def _int8_cases(n_cases=48, seed=4711):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n_cases):
        m = int(rng.choice([1, 7, 33, 100, 256, 300, 777, 1024, 2048, 4096]))
        n = int(rng.integers(8, 4097))
        k = 4 * int(rng.integers(1, 2049)) if i % 2 == 0 else int(rng.integers(1, 8193))   # odd depths too
        out.append((i, m, n, k, bool(rng.integers(0, 2))))
    return out


@pytest.mark.parametrize("case", _int8_cases(), ids=lambda c: f"c{c[0]}-m{c[1]}-n{c[2]}-k{c[3]}-{'b' if c[4] else 'nb'}")
def test_igemmlt_dequant_random_shapes_exact(dev, case):
    import python_src_quants.functional as F
    i, m, n, k, with_bias = case
    rng = np.random.default_rng(77 + i)
    A = rng.integers(-127, 128, size=(m, k), dtype=np.int8)
    B = rng.integers(-127, 128, size=(n, k), dtype=np.int8)
    rs = rng.uniform(0.5, 8.0, m).astype(np.float32)
    cs = rng.uniform(0.5, 8.0, n).astype(np.float32)
    bias = rng.standard_normal(n).astype(np.float16) if with_bias else None
    At, Bt = torch.from_numpy(A).to(dev), torch.from_numpy(B).to(dev)
    out = F.igemmlt_dequant(At, Bt, torch.from_numpy(rs).to(dev), torch.from_numpy(cs).to(dev),
                            bias=torch.from_numpy(bias).to(dev) if with_bias else None)
    C = F.igemm_rowmajor(At, Bt)
    exact = (At.double() @ Bt.double().T).cpu().numpy().astype(np.int64).astype(np.int32)   # |sum| < 2^53: exact
    assert np.array_equal(C.cpu().numpy(), exact)
    exp = ref.mm_dequant(exact, rs, cs, bias)
    assert np.array_equal(out.cpu().numpy().view(np.uint16), np.asarray(exp).view(np.uint16))
