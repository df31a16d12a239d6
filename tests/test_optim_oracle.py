"""CPU checks that pin the optimizer oracle (oracle/optim.py) without a GPU.

* The upstream quantize_2D search (kernel_quant.cpp:840-888 with its code lookup restored, Q21)
  returns exactly what ref.quantize_8bit_dynamic (dQuantize<0>) returns for both dynamic maps.
* The fp32-state oracle tracks torch.optim (Adam, SGD momentum, RMSprop, Adagrad) to fp32 rounding.
* The 8-bit blockwise oracle stays within the reference test's bounds against torch.optim
  (ref:tests_pvc/test_optimizer8bit.py:105-215 protocol, on a smaller tensor).
"""
import numpy as np
import pytest
import torch

from oracle import optim as oref
from oracle import ref


def _dynamic_map(signed):
    import python_src_quants.functional as F
    return F.create_dynamic_map(signed=signed).numpy()


def _quantize_2d_upstream(code, x, signed):
    """quantize_2D<SIGNED> with quadrants = code[63], code[127], code[191] and the code lookup of the
    later steps (the reference writes 0 there, Q21), scalar form."""
    quadrants = [code[63], code[127], code[191]]
    pivot, upper_pivot, lower_pivot = 127, 255, 0
    lower = np.float32(-1.0 if signed else 0.0)
    upper = np.float32(1.0)
    val = quadrants[1]
    local_pivot, offset = 1, 1
    i = 64
    while i > 0:
        if x > val:
            lower_pivot, lower = pivot, val
            pivot += i
            local_pivot += offset
        else:
            upper_pivot, upper = pivot, val
            pivot -= i
            local_pivot -= offset
        val = quadrants[local_pivot] if i >= 64 else code[pivot]
        offset -= 1
        i >>= 1
    if x > val:
        mid = np.float32((upper + val) * np.float32(0.5))
        return upper_pivot if x > mid else pivot
    mid = np.float32((lower + val) * np.float32(0.5))
    return lower_pivot if x < mid else pivot


@pytest.mark.parametrize("signed", [True, False])
def test_quantize_2d_equals_dquantize(signed):
    code = _dynamic_map(signed)
    assert code[255] == 1.0
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.uniform(-1 if signed else 0, 1, 3000).astype(np.float32), code,
                        ((code[1:] + code[:-1]) * np.float32(0.5)).astype(np.float32),
                        np.array([0.0, -0.0, 1.0, 1e-9, -1e-9], np.float32)])
    if not signed:
        x = x[x >= 0]
    got = ref.quantize_8bit_dynamic(code, x)
    exp = np.array([_quantize_2d_upstream(code, np.float32(v), signed) for v in x], np.uint8)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("name", ["adam", "momentum", "rmsprop", "adagrad"])
def test_32bit_oracle_tracks_torch(name):
    torch.manual_seed(0)
    p0 = torch.randn(5000) * 0.1
    tp = p0.clone().requires_grad_(True)
    lr = 1e-3 if name == "adam" else 1e-2
    topt = {"adam": lambda: torch.optim.Adam([tp], lr=lr, eps=1e-8),
            "momentum": lambda: torch.optim.SGD([tp], lr, 0.9),
            "rmsprop": lambda: torch.optim.RMSprop([tp], lr, 0.9, eps=1e-8),
            "adagrad": lambda: torch.optim.Adagrad([tp], lr, eps=1e-10)}[name]()
    b1, b2, eps = {"adam": (0.9, 0.999, 1e-8), "momentum": (0.9, 0.0, 0.0), "rmsprop": (0.9, 0.0, 1e-8),
                   "adagrad": (0.0, 0.0, 1e-10)}[name]
    p = p0.numpy().copy()
    s1 = np.zeros_like(p)
    s2 = np.zeros_like(p) if name == "adam" else None
    for step in range(1, 11):
        g = torch.randn(5000) * 0.01
        tp.grad = g.clone()
        topt.step()
        p, s1, s2 = oref.update_32bit(name, g.numpy(), p, s1, s2, b1, b2, eps, step, lr)
    assert np.allclose(p, tp.detach().numpy(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("name", ["adam", "momentum", "rmsprop"])
def test_8bit_blockwise_oracle_within_reference_bounds(name):
    torch.manual_seed(1)
    n = 64 * 1024
    p1 = (torch.randn(n) * 0.1).requires_grad_(True)
    lr = 1e-3 if name == "adam" else 1e-2
    topt = {"adam": lambda: torch.optim.Adam([p1]), "momentum": lambda: torch.optim.SGD([p1], lr, 0.9),
            "rmsprop": lambda: torch.optim.RMSprop([p1], lr, 0.9)}[name]()
    b1, b2, eps = {"adam": (0.9, 0.999, 1e-8), "momentum": (0.9, 0.0, 0.0), "rmsprop": (0.9, 0.0, 1e-8)}[name]
    code1, code2 = _dynamic_map(True), _dynamic_map(False)
    p2 = p1.detach().numpy().copy()
    c1 = np.zeros(n, np.uint8)
    c2 = np.zeros(n, np.uint8)
    a1 = np.zeros(n // 2048, np.float32)
    a2 = np.zeros(n // 2048, np.float32)
    for step in range(1, 21):
        g = torch.randn(n) * 0.01
        p1.grad = g.clone()
        topt.step()
        p2, c1, c2n, a1, a2n = oref.update_8bit_blockwise(name, g.numpy(), p2, c1, c2, code1, code2, a1, a2, b1, b2,
                                                          eps, step, lr)
        if name == "adam":
            c2, a2 = c2n, a2n
        if step % 10 == 0:
            bad = ~np.isclose(p1.detach().numpy(), p2, rtol=1e-3, atol=1e-5)
            assert bad.sum() <= 5000 * n // (1024 * 1024) + 5
        # the reference's re-sync: our parameters take torch's values, torch's states take our
        # dequantised 8-bit states (ref:tests_pvc/test_optimizer8bit.py:207-212)
        p2 = p1.detach().numpy().copy()
        blk = np.arange(n) // 2048
        st = topt.state[p1]
        key1 = {"adam": "exp_avg", "momentum": "momentum_buffer", "rmsprop": "square_avg"}[name]
        st[key1].copy_(torch.from_numpy((code1[c1] * a1[blk]).astype(np.float32)))
        if name == "adam":
            st["exp_avg_sq"].copy_(torch.from_numpy((code2[c2] * a2[blk]).astype(np.float32)))
