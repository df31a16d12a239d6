"""GPU parity: optimizer updates with 8-bit blockwise and fp32 states.

Bit-exact against the oracle (oracle/optim.py) for every output: the parameter (T bits), the 8-bit
state codes, the per-block absmax and the fp32 states, over several consecutive steps from zero
state, on ragged sizes (a partial last 2048-block), with weight decay, skip_zeros and non-finite
gradients.  The optimizer classes are then checked against torch.optim with the protocol and bounds
of the reference's own test (ref:tests_pvc/test_optimizer8bit.py:105-215).
"""
import zlib

import numpy as np
import pytest
import torch

from helpers import DTYPES, to_numpy, to_torch
from oracle import optim as oref
from oracle import ref

pytestmark = pytest.mark.gpu

NAMES = ["adam", "momentum", "rmsprop", "adagrad", "lion"]
HP = {"adam": (0.9, 0.999, 1e-8, 1e-3), "momentum": (0.9, 0.0, 0.0, 1e-2), "rmsprop": (0.9, 0.0, 1e-8, 1e-2),
      "adagrad": (0.0, 0.0, 1e-10, 1e-2), "lion": (0.9, 0.99, 0.0, 1e-4)}


def _F():
    import python_src_quants.functional as F
    return F


def _rand(rng, n, kind, scale):
    v = (rng.standard_normal(n) * scale).astype(np.float32)
    return ref.cast_out(v, kind)


@pytest.mark.parametrize("kind", ["fp32", "fp16", "bf16"])
@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("case", ["plain", "ragged_wd", "edge"])
def test_8bit_blockwise_vs_oracle(dev, name, kind, case):
    F = _F()
    rng = np.random.default_rng(zlib.crc32(f"{name}-{kind}-{case}".encode()))
    n = {"plain": 3 * 2048, "ragged_wd": 2048 * 5 + 777, "edge": 2048 + 13}[case]
    wd = 0.01 if case == "ragged_wd" else 0.0
    skip = case == "edge" and name != "adam"
    b1, b2, eps, lr = HP[name]
    code1 = F.create_dynamic_map(signed=True)
    code2 = F.create_dynamic_map(signed=False)
    p = _rand(rng, n, kind, 0.1)
    c1 = np.zeros(n, np.uint8)
    c2 = np.zeros(n, np.uint8)
    nb = (n + 2047) // 2048
    a1 = np.zeros(nb, np.float32)
    a2 = np.zeros(nb, np.float32)
    tp = to_torch(p, kind, dev)
    t1 = torch.zeros(n, dtype=torch.uint8, device=dev)
    t2 = torch.zeros(n, dtype=torch.uint8, device=dev) if name == "adam" else None
    ta1 = torch.zeros(nb, device=dev)
    ta2 = torch.zeros(nb, device=dev) if name == "adam" else None
    q1, q2 = code1.to(dev), code2.to(dev)
    for step in range(1, 5):
        g = _rand(rng, n, kind, 0.01)
        if case == "edge":
            g32 = ref.as_f32(g, kind).copy()
            g32[::97] = 0.0                              # skip_zeros candidates / zero gradients
            if name == "adam":
                g32[5] = np.inf
                g32[2048 + 3] = np.nan                    # non-finite gradients leave p unchanged
            g = ref.cast_out(g32, kind)
        tg = to_torch(g, kind, dev)
        F.optimizer_update_8bit_blockwise(name, tg, tp, t1, t2, b1, b2, eps, step, lr, q1, q2 if t2 is not None else None,
                                          ta1, ta2, weight_decay=wd, skip_zeros=skip)
        p, c1, c2n, a1, a2n = oref.update_8bit_blockwise(name, g, p, c1, c2, code1.numpy(), code2.numpy(), a1, a2,
                                                         b1, b2, eps, step, lr, wd, 1.0, skip, kind)
        torch.cuda.synchronize()
        assert np.array_equal(to_numpy(tp, kind).view(np.uint8), np.ascontiguousarray(p).view(np.uint8)), \
            f"param differs at step {step}"
        assert np.array_equal(t1.cpu().numpy(), c1), f"state1 codes differ at step {step}"
        assert np.array_equal(ta1.cpu().numpy().view(np.uint32), a1.view(np.uint32)), f"absmax1 differs at step {step}"
        if name == "adam":
            c2, a2 = c2n, a2n
            assert np.array_equal(t2.cpu().numpy(), c2), f"state2 codes differ at step {step}"
            assert np.array_equal(ta2.cpu().numpy().view(np.uint32), a2.view(np.uint32))


@pytest.mark.parametrize("kind", ["fp32", "fp16", "bf16"])
@pytest.mark.parametrize("name", NAMES)
def test_32bit_vs_oracle(dev, name, kind):
    F = _F()
    rng = np.random.default_rng(7 + NAMES.index(name))
    n = 4096 + 333
    b1, b2, eps, lr = HP[name]
    wd = 0.01
    p = _rand(rng, n, kind, 0.1)
    s1 = np.zeros(n, np.float32)
    s2 = np.zeros(n, np.float32) if name == "adam" else None
    tp = to_torch(p, kind, dev)
    ts1 = torch.zeros(n, device=dev)
    ts2 = torch.zeros(n, device=dev) if name == "adam" else None
    for step in range(1, 4):
        g32 = (rng.standard_normal(n) * 0.01).astype(np.float32)
        g32[::50] = 0.0
        g = ref.cast_out(g32, kind)
        F.optimizer_update_32bit(name, to_torch(g, kind, dev), tp, ts1, b1, eps, step, lr, ts2, b2, wd,
                                 skip_zeros=(step == 2))
        p, s1, s2 = oref.update_32bit(name, g, p, s1, s2, b1, b2, eps, step, lr, wd, 1.0, step == 2, kind)
        torch.cuda.synchronize()
        assert np.array_equal(to_numpy(tp, kind).view(np.uint8), np.ascontiguousarray(p).view(np.uint8))
        assert np.array_equal(ts1.cpu().numpy().view(np.uint32), s1.view(np.uint32))
        if name == "adam":
            assert np.array_equal(ts2.cpu().numpy().view(np.uint32), s2.view(np.uint32))


def _most_close(a, b, atol, rtol, max_error_count):
    """ref:tests_pvc/helpers assert_most_approx_close."""
    idx = torch.isclose(a, b, rtol=rtol, atol=atol)
    assert (idx == 0).sum().item() <= max_error_count


@pytest.mark.parametrize("gtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("optim_name", ["adam8bit_blockwise", "momentum8bit_blockwise", "rmsprop8bit_blockwise",
                                        "adam", "momentum", "rmsprop"])
def test_optimizer_vs_torch(dev, gtype, optim_name):
    """The reference test's protocol (ref:tests_pvc/test_optimizer8bit.py:105-215): step both, compare
    the parameters every 10 steps with its bounds, then re-sync the torch copy to ours."""
    import python_src_quants as bnb
    F = _F()
    if gtype == torch.bfloat16 and optim_name not in ("adam8bit_blockwise", "adam"):
        pytest.skip("the reference runs bf16 only for Adam")
    make = {
        "adam8bit_blockwise": (torch.optim.Adam, lambda ps: bnb.optim.Adam8bit(ps, block_wise=True)),
        "momentum8bit_blockwise": (lambda ps: torch.optim.SGD(ps, 0.01, 0.9),
                                   lambda ps: bnb.optim.SGD8bit(ps, 0.01, 0.9, block_wise=True)),
        "rmsprop8bit_blockwise": (lambda ps: torch.optim.RMSprop(ps, 0.01, 0.9),
                                  lambda ps: bnb.optim.RMSprop8bit(ps, 0.01, 0.9, block_wise=True)),
        "adam": (torch.optim.Adam, bnb.optim.Adam),
        "momentum": (lambda ps: torch.optim.SGD(ps, 0.01, 0.9), lambda ps: bnb.optim.SGD(ps, 0.01, 0.9)),
        "rmsprop": (lambda ps: torch.optim.RMSprop(ps, 0.01, 0.9), lambda ps: bnb.optim.RMSprop(ps, 0.01, 0.9)),
    }[optim_name]
    torch.manual_seed(0)
    p1 = torch.randn(1024, 1024, device=dev, dtype=gtype) * 0.1
    p2 = p1.clone()
    p1 = p1.float()
    topt, bopt = make[0]([p1]), make[1]([p2])
    patol, prtol = (1e-4, 1e-2) if gtype == torch.bfloat16 else (1e-5, 1e-3)
    for i in range(50):
        g = torch.randn(1024, 1024, device=dev, dtype=gtype) * 0.01
        p1.grad = g.clone().float()
        p2.grad = g.clone()
        bopt.step()
        topt.step()
        if i % 10 == 0 and i > 0:
            _most_close(p1, p2.float(), patol, prtol, max_error_count=5000)
        # the reference's re-sync: our parameters take torch's values and torch's states take ours
        # (dequantised for 8-bit states)
        p1.data = p1.data.to(gtype).float()
        p2.copy_(p1.data)
        st, ts = bopt.state[p2], topt.state[p1]
        names = {"adam": ["exp_avg", "exp_avg_sq"], "momentum": ["momentum_buffer"],
                 "rmsprop": ["square_avg"]}[optim_name.replace("8bit_blockwise", "")]
        for j, key in enumerate(names):
            s = st[f"state{j + 1}"]
            if s.dtype == torch.uint8:
                s = F.dequantize_blockwise(s, absmax=st[f"absmax{j + 1}"], code=st[f"qmap{j + 1}"], blocksize=2048)
            ts[key].copy_(s.view_as(ts[key]).float())


def test_state_dict_roundtrip(dev, tmp_path):
    """Save / load keeps the 8-bit state bit for bit (ref:tests_pvc/test_optimizer8bit.py:175-200)."""
    import python_src_quants as bnb
    torch.manual_seed(1)
    p = torch.nn.Parameter(torch.randn(4096 + 100, device=dev) * 0.1)
    opt = bnb.optim.Adam8bit([p])
    for _ in range(3):
        p.grad = torch.randn_like(p) * 0.01
        opt.step()
    path = tmp_path / "opt.pt"
    torch.save(opt.state_dict(), path)
    opt2 = bnb.optim.Adam8bit([p])
    opt2.load_state_dict(torch.load(path, weights_only=True))
    for k in ("state1", "state2", "qmap1", "qmap2", "absmax1", "absmax2"):
        assert torch.equal(opt.state[p][k], opt2.state[p][k]), k
    assert opt2.state[p]["state1"].dtype == torch.uint8
    g = torch.randn_like(p) * 0.01
    q = p.detach().clone()
    p.grad = g.clone()
    opt.step()
    a = p.detach().clone()
    p.data.copy_(q)
    p.grad = g.clone()
    opt2.step()
    assert torch.equal(a, p.detach())


def test_small_params_use_fp32_state_and_training_runs(dev):
    """min_8bit_size routing (ref:optim/optimizer.py:432-434) and a Linear8bitLt + Adam8bit training
    loop (ref:tests_pvc/test_simple_nn.py) whose loss decreases."""
    import python_src_quants as bnb
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(784, 256), torch.nn.ReLU(), torch.nn.Linear(256, 10)).to(dev)
    opt = bnb.optim.Adam8bit(model.parameters(), lr=1e-3)
    x = torch.randn(256, 784, device=dev)
    y = torch.randint(0, 10, (256,), device=dev)
    losses = []
    for _ in range(30):
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < 0.5 * losses[0]
    st = opt.state[model[0].weight]
    assert st["state1"].dtype == torch.uint8 and st["absmax1"].numel() == (784 * 256 + 2047) // 2048
    assert opt.state[model[0].bias]["state1"].dtype == torch.float32      # 256 < min_8bit_size


def test_global_manager_override_changes_state_kind(dev):
    """GlobalOptimManager: a 32-bit optimizer with one parameter overridden to 8-bit state keeps uint8
    blockwise state for that parameter only, and its update equals Adam8bit's on the same input."""
    import python_src_quants as bnb
    mng = bnb.optim.GlobalOptimManager.get_instance()
    mng.initialize()
    torch.manual_seed(3)
    p1, p2 = (torch.nn.Parameter(torch.randn(8192, device=dev) * 0.1) for _ in range(2))
    ref = torch.nn.Parameter(p2.detach().clone())
    mng.override_config(p2, "optim_bits", 8)
    mng.register_parameters([p1, p2])
    opt = bnb.optim.Adam([p1, p2], lr=1e-3)
    opt_ref = bnb.optim.Adam8bit([ref], lr=1e-3)
    for _ in range(3):
        g = torch.randn_like(p2) * 0.01
        p1.grad, p2.grad, ref.grad = torch.randn_like(p1) * 0.01, g.clone(), g.clone()
        opt.step()
        opt_ref.step()
    assert opt.state[p1]["state1"].dtype == torch.float32
    assert opt.state[p2]["state1"].dtype == torch.uint8
    assert torch.equal(p2.detach(), ref.detach())
    mng.initialize()
