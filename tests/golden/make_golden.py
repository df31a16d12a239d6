"""Generate the committed golden vectors under tests/golden/ from the CPU oracle.

The reference ships no golden vectors for this path and may not be executed here
(SURVEY.md §8c), so these fixtures are produced by the oracle restatement (oracle/ref.py),
whose constants are pinned against the reference source in tests/test_oracle_pins.py.
They freeze the oracle's outputs (regression) and are the inputs/expected outputs the
GPU parity tests check the HIP kernels against.

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import ref  # noqa: E402
from oracle.maps import create_dynamic_map  # noqa: E402


def _input(rng, n, dtype):
    x = (rng.standard_normal(n) * 1.5).astype(np.float32)
    # edge values: exact thresholds/values, zeros, +-0, huge/small magnitudes
    if n >= 20:
        x[:16] = ref.NF4_THRESHOLDS[np.arange(16) % 15]
        x[16:20] = [0.0, -0.0, 1e-30, -1e-30]
    if dtype == "bf16":
        return ref.f32_to_bf16_bits(x)
    if dtype == "fp16":
        return x.astype(np.float16)
    return x


def quant_cases():
    rng = np.random.default_rng(1234)
    code = create_dynamic_map()
    out = {"dynamic_code": code}
    cases = []
    for dtype in ("fp32", "fp16", "bf16"):
        for qtype in ("nf4", "fp4", "8bit"):
            for bs, n in ((64, 64 * 7 + 33), (128, 1000), (256, 513), (4096, 4096 + 77), (64, 1)):
                cases.append((dtype, qtype, bs, n))
    for i, (dtype, qtype, bs, n) in enumerate(cases):
        a = _input(rng, n, dtype)
        if n > 200:
            a[128:192] = 0          # an all-zero block (bs=64 case) / zero run
        xf = ref.as_f32(a, dtype)
        absmax, q = ref.quantize_blockwise(xf, bs, qtype, code=code)
        deq = {}
        for od in ("fp32", "fp16", "bf16"):
            deq[od] = ref.dequantize_blockwise(q, absmax, bs, n, qtype, od, code=code)
        key = f"q{i}"
        out[f"{key}_meta"] = np.array([["fp32", "fp16", "bf16"].index(dtype), ["nf4", "fp4", "8bit"].index(qtype), bs, n])
        out[f"{key}_in"] = a
        out[f"{key}_absmax"] = absmax
        out[f"{key}_q"] = q
        for od, v in deq.items():
            out[f"{key}_deq_{od}"] = v
    out["n_quant_cases"] = np.array(len(cases))
    return out


def gemv_case():
    rng = np.random.default_rng(7)
    N, K, bs = 96, 256, 64
    w = (rng.standard_normal(N * K) * 0.02).astype(np.float32)
    absmax, q = ref.quantize_blockwise(w, bs, "nf4")
    x = ref.f32_to_bf16_bits(rng.standard_normal(K).astype(np.float32))
    y = ref.gemv_4bit(ref.bf16_bits_to_f32(x), q, absmax, N, K, bs, ref.nf4_table())
    return {"gemv_w": w, "gemv_q": q, "gemv_absmax": absmax, "gemv_x": x, "gemv_y": y,
            "gemv_meta": np.array([N, K, bs])}


def int8_case():
    rng = np.random.default_rng(11)
    A = (rng.standard_normal((130, 70)) * 3).astype(np.float16)
    A[5, :] = 0                 # all-zero row -> rowStat 0 -> NaN scale -> 0
    rs, cs, _ = ref.colrow_absmax(A)
    orow, ocol = ref.double_quant(A, rs, cs)
    Ai = rng.integers(-127, 128, size=(64, 96), dtype=np.int8)
    Bi = rng.integers(-127, 128, size=(40, 96), dtype=np.int8)
    C = ref.igemmlt(Ai, Bi)
    rstat = rng.uniform(0.5, 2, 64).astype(np.float32)
    cstat = rng.uniform(0.5, 2, 40).astype(np.float32)
    bias = rng.standard_normal(40).astype(np.float16)
    D = ref.mm_dequant(C, rstat, cstat, bias)
    out = {"dq_A": A, "dq_rs": rs, "dq_cs": cs, "dq_row": orow, "dq_col": ocol,
           "ig_A": Ai, "ig_B": Bi, "ig_C": C, "ig_rstat": rstat, "ig_cstat": cstat, "ig_bias": bias, "ig_D": D}
    for fmt in ("col32", "col_turing", "col_ampere"):
        out[f"tf_{fmt}"] = ref.transform(Ai, fmt)
        out[f"tfT_{fmt}"] = ref.transform(Ai, fmt, transpose=True)
    return out


def cpu_path_case():
    rng = np.random.default_rng(5)
    code = create_dynamic_map()
    A = rng.standard_normal(1000).astype(np.float32)
    absmax, q, code_after = ref.quantize_cpu(code, A, 64)
    deq = ref.dequantize_cpu(code_after, q, absmax, 64)
    return {"cpu_A": A, "cpu_absmax": absmax, "cpu_q": q, "cpu_code_after": code_after, "cpu_deq": deq}


def main():
    data = {}
    data.update(quant_cases())
    data.update(gemv_case())
    data.update(int8_case())
    data.update(cpu_path_case())
    path = os.path.join(HERE, "golden_v1.npz")
    np.savez_compressed(path, **data)
    print(f"wrote {path}: {os.path.getsize(path)} bytes, {len(data)} arrays")


if __name__ == "__main__":
    main()
