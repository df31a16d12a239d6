"""Host logic of the optimizer classes (no GPU): GlobalOptimManager overrides and
Optimizer8bit.load_state_dict's dtype rules (behaviour of ref:optim/optimizer.py:24-110, 147-215, 217-226)."""
import pytest
import torch


def _bnb():
    import python_src_quants as bnb
    return bnb


def _fresh_manager():
    mng = _bnb().optim.GlobalOptimManager.get_instance()
    mng.initialize()
    return mng


def test_manager_is_a_singleton_and_not_constructible():
    GOM = _bnb().optim.GlobalOptimManager
    assert GOM.get_instance() is GOM.get_instance()
    with pytest.raises(RuntimeError):
        GOM()


def test_override_before_registration_reaches_get_config():
    bnb = _bnb()
    mng = _fresh_manager()
    p1, p2, p3 = (torch.nn.Parameter(torch.randn(64, 64)) for _ in range(3))
    mng.override_config(p3, "optim_bits", 8)
    mng.override_config([p1, p3], key_value_dict={"eps": 1e-6, "lr": 5e-4})
    mng.register_parameters([p1, p2, p3])
    opt = bnb.optim.Adam([p1, p2, p3], lr=1e-3, optim_bits=32)
    group = opt.param_groups[0]
    c1, c2, c3 = (opt.get_config(0, i, group) for i in range(3))
    assert c1["optim_bits"] == 32 and c1["eps"] == 1e-6 and c1["lr"] == 5e-4
    assert c2["optim_bits"] == 32 and c2["eps"] == group["eps"] and c2["lr"] == 1e-3
    assert c3["optim_bits"] == 8 and c3["eps"] == 1e-6
    assert mng.uses_config_override
    # param groups given as dicts register by (group, position)
    mng = _fresh_manager()
    mng.override_config(p2, "betas", (0.8, 0.9))
    mng.register_parameters([{"params": [p1]}, {"params": [p3, p2]}])
    assert set(mng.index2config) == {(1, 1)}
    with pytest.raises(ValueError):
        mng.override_config(p1, "eps", 1e-5, key_value_dict={"lr": 1.0})


def test_module_override_resolves_at_first_lookup():
    bnb = _bnb()
    mng = _fresh_manager()
    model = torch.nn.Sequential(torch.nn.Linear(8, 8), torch.nn.Linear(8, 4))
    mng.register_module_override(model[1], "weight", {"optim_bits": 32, "lr": 7e-3})
    opt = bnb.optim.Adam8bit(model.parameters(), lr=1e-3)
    opt.check_overrides()
    slot = next(i for i, p in enumerate(opt.param_groups[0]["params"]) if p is model[1].weight)
    cfg = opt.get_config(0, slot, opt.param_groups[0])
    assert cfg["optim_bits"] == 32 and cfg["lr"] == 7e-3
    other = opt.get_config(0, 0, opt.param_groups[0])
    assert other["optim_bits"] == 8 and other["lr"] == 1e-3


def test_load_state_dict_keeps_8bit_state_and_casts_the_rest():
    bnb = _bnb()
    _fresh_manager()
    p = torch.nn.Parameter(torch.randn(4096, dtype=torch.float16))
    q = torch.nn.Parameter(torch.randn(16, dtype=torch.float16))
    opt = bnb.optim.Adam8bit([p, q], lr=2e-3, betas=(0.8, 0.95))
    opt.state[p] = {"step": 3, "state1": torch.randint(0, 255, (4096,), dtype=torch.uint8),
                    "qmap1": torch.linspace(-1, 1, 256), "absmax1": torch.rand(2),
                    "extra": torch.randn(4), "nested": [torch.randn(2), (torch.randn(1),)]}
    sd = opt.state_dict()
    opt2 = bnb.optim.Adam8bit([p, q], lr=1.0)
    opt2.load_state_dict(sd)
    st = opt2.state[p]
    assert st["step"] == 3
    assert st["state1"].dtype == torch.uint8 and torch.equal(st["state1"], opt.state[p]["state1"])
    assert st["qmap1"].dtype == torch.float32 and st["absmax1"].dtype == torch.float32   # non-castable keys
    assert st["extra"].dtype == torch.float16                                           # cast to the parameter
    assert st["nested"][0].dtype == torch.float16 and isinstance(st["nested"][1], tuple)
    assert opt2.param_groups[0]["lr"] == 2e-3 and tuple(opt2.param_groups[0]["betas"]) == (0.8, 0.95)
    assert opt2.param_groups[0]["params"][0] is p
    assert q not in opt2.state
    with pytest.raises(ValueError):
        bnb.optim.Adam8bit([p], lr=1.0).load_state_dict(sd)
    bad = opt.state_dict()
    bad["param_groups"].append(dict(bad["param_groups"][0]))
    with pytest.raises(ValueError):
        opt2.load_state_dict(bad)
