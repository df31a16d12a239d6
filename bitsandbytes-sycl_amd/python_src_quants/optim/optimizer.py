"""8-bit / 32-bit state optimizers, mirroring ref:python_src_quants/optim/optimizer.py.

Optimizer8bit / Optimizer2State / Optimizer1State keep the reference's constructor arguments, state
keys (step, state1, state2, qmap1, qmap2, absmax1, absmax2), GlobalOptimManager overrides and
state_dict round trip.  Per parameter the update is one HIP launch:
  * 8-bit blockwise states (optim_bits=8, block_wise=True, numel >= min_8bit_size):
    F.optimizer_update_8bit_blockwise -> c<name>_8bit_blockwise_grad_<T>;
  * fp32 states otherwise: F.optimizer_update_32bit -> c<name>32bit_grad_<T>.
Not provided by this backend (they raise NotImplementedError): the non-blockwise 8-bit path
(global max, kOptimizerStatic8bit2State), percentile clipping, max_unorm and paged state.
"""
from __future__ import annotations

from collections import defaultdict
from copy import deepcopy

import torch

from .. import functional as F


class MockArgs:
    """Attribute view of a config dict (the reference's optimizers read ``self.args.<key>``)."""

    def __init__(self, initial_data):
        self.__dict__.update(initial_data)


class GlobalOptimManager:
    """Process-wide registry of per-parameter optimizer settings (behaviour of ref:optim/optimizer.py:24-110).

    Overrides are recorded against the parameter object (``id(p)``) while a model is being built --
    ``override_config`` directly, ``register_module_override`` by (module, attribute) resolved at the
    optimizer's first step -- and re-keyed by (group index, position in group) when parameters are
    registered, which is the key ``Optimizer8bit.get_config`` looks up.
    """
    _instance = None

    def __init__(self):
        raise RuntimeError("Call get_instance() instead")

    @classmethod
    def get_instance(cls):
        if cls._instance is None:
            manager = object.__new__(cls)
            manager.initialize()
            cls._instance = manager
        return cls._instance

    def initialize(self):
        self.pid2config = {}                     # id(parameter) -> {setting: value}
        self.index2config = {}                   # (group index, parameter index) -> the same dict
        self.module_weight_config_triple = []    # (module, attribute name, settings), resolved lazily
        self.optimizer = None
        self.uses_config_override = False

    @staticmethod
    def _param_groups(params):
        params = list(params)
        if params and isinstance(params[0], dict):
            return params
        return [{"params": params}]

    def register_parameters(self, params):
        """Attach the id()-keyed overrides to the (group, position) slots of ``params``."""
        for gindex, group in enumerate(self._param_groups(params)):
            for pindex, p in enumerate(group["params"]):
                settings = self.pid2config.get(id(p))
                if settings is not None:
                    self.index2config[(gindex, pindex)] = settings

    def override_config(self, parameters, key=None, value=None, key_value_dict=None):
        """Override settings for one tensor or an iterable of tensors: ``key``/``value`` for one setting,
        ``key_value_dict`` for several (not both)."""
        if key is not None and value is not None:
            if key_value_dict is not None:
                raise ValueError("pass either key/value or key_value_dict, not both")
            key_value_dict = {key: value}
        self.uses_config_override = True
        if key_value_dict is None:
            return
        targets = [parameters] if isinstance(parameters, torch.Tensor) else parameters
        for p in targets:
            self.pid2config.setdefault(id(p), {}).update(key_value_dict)

    def register_module_override(self, module, param_name, config):
        """Override settings for ``getattr(module, param_name)``, looked up when the optimizer first steps."""
        self.module_weight_config_triple.append((module, param_name, config))


class Optimizer8bit(torch.optim.Optimizer):
    """Base class (ref:optim/optimizer.py:113-343)."""

    def __init__(self, params, defaults, optim_bits=32, is_paged=False):
        super().__init__(params, defaults)
        if is_paged:
            raise NotImplementedError("paged optimizer state is not supported by the MI355X backend")
        self.initialized = False
        self.name2qmap = {}
        self.is_paged = is_paged
        self.mng = GlobalOptimManager.get_instance()
        self.non_castable_tensor_keys = {"qmap1", "qmap2", "max1", "max2", "new_max1", "new_max2", "state1",
                                         "state2", "gnorm_vec", "absmax1", "absmax2", "unorm_vec"}
        if optim_bits == 8:
            self.fill_qmap()

    def fill_qmap(self):
        self.name2qmap["dynamic"] = F.create_dynamic_map(signed=True)
        self.name2qmap["udynamic"] = F.create_dynamic_map(signed=False)

    def __setstate__(self, state):
        super().__setstate__(state)

    def load_state_dict(self, state_dict):
        """Restore a saved state (behaviour of ref:optim/optimizer.py:147-215).  Unlike
        torch.optim.Optimizer's version, 8-bit state keeps its dtype: tensors named in
        ``non_castable_tensor_keys`` only move to the parameter's device; other floating tensors take the
        parameter's dtype; uint8 tensors are left as they are."""
        saved = deepcopy(state_dict)
        groups, saved_groups = self.param_groups, saved["param_groups"]
        if len(groups) != len(saved_groups):
            raise ValueError("loaded state dict has a different number of parameter groups")
        for group, saved_group in zip(groups, saved_groups):
            if len(group["params"]) != len(saved_group["params"]):
                raise ValueError("loaded state dict contains a parameter group that doesn't match the size of "
                                 "optimizer's group")
        param_of = {}                            # saved parameter id -> live parameter
        for group, saved_group in zip(groups, saved_groups):
            param_of.update(zip(saved_group["params"], group["params"]))
        state = defaultdict(dict)
        for saved_id, value in saved["state"].items():
            p = param_of.get(saved_id)
            if p is None:
                state[saved_id] = value
            else:
                state[p] = self._restore_state_value(p, value)
        param_groups = [dict(saved_group, params=group["params"]) for group, saved_group in zip(groups, saved_groups)]
        self.__setstate__({"state": state, "param_groups": param_groups})

    def _restore_state_value(self, p, value, key=None):
        if isinstance(value, torch.Tensor):
            if key in self.non_castable_tensor_keys:
                return value.to(p.device)
            if p.is_floating_point() and value.dtype != torch.uint8:
                return value.to(p.dtype)
            return value
        if isinstance(value, dict):
            return {k: self._restore_state_value(p, v, k) for k, v in value.items()}
        if isinstance(value, (list, tuple)):
            return type(value)(self._restore_state_value(p, v) for v in value)
        return value

    def to_gpu(self):
        for group in self.param_groups:
            for p in group["params"]:
                if p in self.state:
                    for k, v in self.state[p].items():
                        if isinstance(v, torch.Tensor):
                            self.state[p][k] = v.to(p.device)

    def check_overrides(self):
        """Resolve register_module_override entries: the first slot holding that module attribute's tensor
        takes the settings."""
        slots = {}
        for gindex, group in enumerate(self.param_groups):
            for pindex, p in enumerate(group["params"]):
                slots.setdefault(id(p), (gindex, pindex))
        for module, attr, config in self.mng.module_weight_config_triple:
            target = getattr(module, attr)
            assert target is not None
            slot = slots.get(id(target))
            if slot is not None:
                self.mng.pid2config[id(target)] = config
                self.mng.index2config[slot] = config

    @torch.no_grad()
    def step(self, closure=None):
        """One optimisation step over every parameter with a gradient (ref:optim/optimizer.py:244-287).
        Launches are stream-ordered; unlike the reference there is no device synchronise per parameter."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if not self.initialized:
            self.check_overrides()
            self.to_gpu()
            self.initialized = True
        for gindex, group in enumerate(self.param_groups):
            for pindex, p in enumerate(group["params"]):
                if p.grad is None:
                    continue
                state = self.state[p]
                if len(state) == 0:
                    self.init_state(group, p, gindex, pindex)
                self.update_step(group, p, gindex, pindex)
        return loss

    def get_config(self, gindex, pindex, group):
        config = {"betas": group["betas"], "eps": group["eps"], "weight_decay": group["weight_decay"],
                  "lr": group["lr"], "optim_bits": self.args.optim_bits, "min_8bit_size": self.args.min_8bit_size,
                  "percentile_clipping": self.args.percentile_clipping, "block_wise": self.args.block_wise,
                  "max_unorm": self.args.max_unorm, "skip_zeros": self.args.skip_zeros}
        if (gindex, pindex) in self.mng.index2config:
            config.update(self.mng.index2config[(gindex, pindex)])
        return config

    def init_state(self, group, p, gindex, pindex):
        raise NotImplementedError("init_state method needs to be overridden")

    def update_step(self, group, p, gindex, pindex):
        raise NotImplementedError("The update_step method needs to be overridden")

    # ---- shared helpers of the two concrete bases
    def _state_dtype(self, config, p):
        if config["optim_bits"] == 32:
            dtype = torch.float32
        elif config["optim_bits"] == 8:
            dtype = torch.uint8
        else:
            raise NotImplementedError(f'Amount of optimizer bits not supported: {config["optim_bits"]}')
        if p.numel() < config["min_8bit_size"]:
            dtype = torch.float32
        if dtype == torch.uint8 and not config["block_wise"]:
            raise NotImplementedError("non-blockwise 8-bit optimizer state is not supported by the MI355X backend "
                                      "(use block_wise=True)")
        if config["percentile_clipping"] < 100:
            raise NotImplementedError("percentile_clipping < 100 is not supported by the MI355X backend")
        if config["max_unorm"] > 0.0:
            raise NotImplementedError("max_unorm > 0 is not supported by the MI355X backend")
        return dtype

    def _qmaps(self, p):
        if "dynamic" not in self.name2qmap:
            self.fill_qmap()
        self.name2qmap["dynamic"] = self.name2qmap["dynamic"].to(p.device)
        self.name2qmap["udynamic"] = self.name2qmap["udynamic"].to(p.device)

    @staticmethod
    def _blocks(p):
        n = p.numel()
        return n // 2048 + (1 if n % 2048 > 0 else 0)


def _make_args(optim_bits, min_8bit_size, percentile_clipping, block_wise, max_unorm, skip_zeros):
    return MockArgs({"optim_bits": optim_bits, "min_8bit_size": min_8bit_size,
                     "percentile_clipping": percentile_clipping, "block_wise": block_wise, "max_unorm": max_unorm,
                     "skip_zeros": skip_zeros})


def _check_hparams(lr, eps, betas, weight_decay):
    if not 0.0 <= lr:
        raise ValueError(f"Invalid learning rate: {lr}")
    if not 0.0 <= eps:
        raise ValueError(f"Invalid epsilon value: {eps}")
    for i in range(len(betas)):
        if not 0.0 <= betas[i] < 1.0:
            raise ValueError(f"Invalid beta parameter at index {i}: {betas[i]}")
    if not 0.0 <= weight_decay:
        raise ValueError(f"Invalid weight_decay value: {weight_decay}")


class Optimizer2State(Optimizer8bit):
    """Two-state optimizers (Adam/AdamW), ref:optim/optimizer.py:346-539."""

    def __init__(self, optimizer_name, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 optim_bits=32, args=None, min_8bit_size=4096, percentile_clipping=100, block_wise=True,
                 max_unorm=0.0, skip_zeros=False, is_paged=False):
        if isinstance(betas, str):
            betas = [float(b) for b in betas.replace("(", "").replace(")", "").strip().split(",")]
        _check_hparams(lr, eps, betas, weight_decay)
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults, optim_bits, is_paged)
        self.args = args if args is not None else _make_args(optim_bits, min_8bit_size, percentile_clipping,
                                                             block_wise, max_unorm, skip_zeros)
        self.optimizer_name = optimizer_name

    @torch.no_grad()
    def init_state(self, group, p, gindex, pindex):
        config = self.get_config(gindex, pindex, group)
        dtype = self._state_dtype(config, p)
        state = self.state[p]
        state["step"] = 0
        if dtype == torch.float32:
            state["state1"] = torch.zeros_like(p, dtype=torch.float32)
            state["state2"] = torch.zeros_like(p, dtype=torch.float32)
        else:
            self._qmaps(p)
            state["state1"] = torch.zeros_like(p, dtype=torch.uint8)
            state["qmap1"] = self.name2qmap["dynamic"]
            state["state2"] = torch.zeros_like(p, dtype=torch.uint8)
            state["qmap2"] = self.name2qmap["udynamic"]
            blocks = self._blocks(p)
            state["absmax1"] = torch.zeros((blocks,), dtype=torch.float32, device=p.device)
            state["absmax2"] = torch.zeros((blocks,), dtype=torch.float32, device=p.device)

    @torch.no_grad()
    def update_step(self, group, p, gindex, pindex):
        p.data = p.data.contiguous()
        p.grad = p.grad.contiguous()
        state = self.state[p]
        grad = p.grad
        config = self.get_config(gindex, pindex, group)
        state["step"] += 1
        step = state["step"]
        if state["state1"].dtype == torch.float:
            F.optimizer_update_32bit(self.optimizer_name, grad, p, state["state1"], config["betas"][0],
                                     config["eps"], step, config["lr"], state["state2"], config["betas"][1],
                                     config["weight_decay"], 1.0, None, max_unorm=config["max_unorm"],
                                     skip_zeros=config["skip_zeros"])
        else:
            F.optimizer_update_8bit_blockwise(self.optimizer_name, grad, p, state["state1"], state["state2"],
                                              config["betas"][0], config["betas"][1], config["eps"], step,
                                              config["lr"], state["qmap1"], state["qmap2"], state["absmax1"],
                                              state["absmax2"], config["weight_decay"], gnorm_scale=1.0,
                                              skip_zeros=config["skip_zeros"])


class Optimizer1State(Optimizer8bit):
    """One-state optimizers (SGD momentum, RMSprop, Adagrad, Lion), ref:optim/optimizer.py:577-782."""

    def __init__(self, optimizer_name, params, lr=1e-3, betas=(0.9, 0.0), eps=1e-8, weight_decay=0.0,
                 optim_bits=32, args=None, min_8bit_size=4096, percentile_clipping=100, block_wise=True,
                 max_unorm=0.0, skip_zeros=False, is_paged=False):
        _check_hparams(lr, eps, betas, weight_decay)
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults, optim_bits, is_paged)
        self.args = args if args is not None else _make_args(optim_bits, min_8bit_size, percentile_clipping,
                                                             block_wise, max_unorm, skip_zeros)
        self.optimizer_name = optimizer_name

    @torch.no_grad()
    def init_state(self, group, p, gindex, pindex):
        config = self.get_config(gindex, pindex, group)
        dtype = self._state_dtype(config, p)
        state = self.state[p]
        state["step"] = 0
        if dtype == torch.float32:
            state["state1"] = torch.zeros_like(p, dtype=torch.float32)
        else:
            self._qmaps(p)
            state["state1"] = torch.zeros_like(p, dtype=torch.uint8)
            state["qmap1"] = self.name2qmap["dynamic"]
            state["absmax1"] = torch.zeros((self._blocks(p),), dtype=torch.float32, device=p.device)

    @torch.no_grad()
    def update_step(self, group, p, gindex, pindex):
        p.data = p.data.contiguous()
        p.grad = p.grad.contiguous()
        state = self.state[p]
        grad = p.grad
        config = self.get_config(gindex, pindex, group)
        state["step"] += 1
        step = state["step"]
        if state["state1"].dtype == torch.float:
            F.optimizer_update_32bit(self.optimizer_name, grad, p, state["state1"], config["betas"][0],
                                     config["eps"], step, config["lr"], None, config["betas"][1],
                                     config["weight_decay"], 1.0, None, max_unorm=config["max_unorm"],
                                     skip_zeros=config["skip_zeros"])
        else:
            F.optimizer_update_8bit_blockwise(self.optimizer_name, grad, p, state["state1"], None,
                                              config["betas"][0], config["betas"][1], config["eps"], step,
                                              config["lr"], state["qmap1"], None, state["absmax1"], None,
                                              config["weight_decay"], gnorm_scale=1.0,
                                              skip_zeros=config["skip_zeros"])
