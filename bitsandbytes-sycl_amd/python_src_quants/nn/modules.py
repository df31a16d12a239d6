"""4-bit and 8-bit linear layers (mirrors ref:python_src_quants/nn/modules.py:212-821) on ROCm."""
from __future__ import annotations

import copy
from typing import Any, Dict, Optional, TypeVar
import warnings

import torch
from torch import nn

from .. import functional as F
from ..autograd._functions import MatmulLtState, matmul, matmul_4bit
from ..functional import QuantState
from ..utils import INVERSE_LINEAR_8BIT_WEIGHTS_FORMAT_MAPPING, LINEAR_8BIT_WEIGHTS_FORMAT_MAPPING

T = TypeVar("T", bound="torch.nn.Module")


class Params4bit(torch.nn.Parameter):
    """Packed 4-bit weight parameter; quantised on the first move to a GPU (ref:nn/modules.py:212-343)."""

    def __new__(cls, data: Optional[torch.Tensor] = None, requires_grad=False, quant_state: Optional[QuantState] = None,
                blocksize: int = 64, compress_statistics: bool = True, quant_type: str = "fp4",
                quant_storage: torch.dtype = torch.uint8, module: Optional["Linear4bit"] = None,
                bnb_quantized: bool = False) -> "Params4bit":
        if data is None:
            data = torch.empty(0)
        self = torch.Tensor._make_subclass(cls, data, requires_grad)
        self.blocksize = blocksize
        self.compress_statistics = compress_statistics
        self.quant_type = quant_type
        self.quant_state = quant_state
        self.quant_storage = quant_storage
        self.bnb_quantized = bnb_quantized
        self.data = data
        self.module = module
        return self

    def __getstate__(self):
        state = self.__dict__.copy()
        state["data"] = self.data
        state["requires_grad"] = self.requires_grad
        return state

    def __setstate__(self, state):
        self.requires_grad = state["requires_grad"]
        self.blocksize = state["blocksize"]
        self.compress_statistics = state["compress_statistics"]
        self.quant_type = state["quant_type"]
        self.quant_state = state["quant_state"]
        self.data = state["data"]
        self.quant_storage = state["quant_storage"]
        self.bnb_quantized = state["bnb_quantized"]
        self.module = state["module"]

    def __deepcopy__(self, memo):
        new_instance = type(self).__new__(type(self))
        state = self.__getstate__()
        new_instance.__setstate__(state)
        new_instance.quant_state = copy.deepcopy(state["quant_state"])
        new_instance.data = copy.deepcopy(state["data"])
        return new_instance

    def __copy__(self):
        new_instance = type(self).__new__(type(self))
        new_instance.__setstate__(self.__getstate__())
        return new_instance

    @classmethod
    def from_prequantized(cls, data: torch.Tensor, quantized_stats: Dict[str, Any], requires_grad: bool = False,
                          device="cuda", **kwargs) -> "Params4bit":
        self = torch.Tensor._make_subclass(cls, data.to(device))
        self.requires_grad = requires_grad
        self.quant_state = QuantState.from_dict(qs_dict=quantized_stats, device=device)
        self.blocksize = self.quant_state.blocksize
        self.compress_statistics = self.quant_state.nested
        self.quant_type = self.quant_state.quant_type
        self.bnb_quantized = True
        self.quant_storage = data.dtype
        self.module = None
        return self

    def _quantize(self, device):
        w = self.data.contiguous().to(device)
        w_4bit, quant_state = F.quantize_4bit(w, blocksize=self.blocksize, compress_statistics=self.compress_statistics,
                                              quant_type=self.quant_type, quant_storage=self.quant_storage)
        self.data = w_4bit
        self.quant_state = quant_state
        if self.module is not None:
            self.module.quant_state = quant_state
        self.bnb_quantized = True
        return self

    def cuda(self, device=None, non_blocking: bool = False):
        return self.to(device="cuda" if device is None else device, non_blocking=non_blocking)

    def to(self, *args, **kwargs):
        device, dtype, non_blocking, _ = torch._C._nn._parse_to(*args, **kwargs)
        if device is not None and device.type == "cuda" and not self.bnb_quantized:
            return self._quantize(device)
        if self.quant_state is not None:
            self.quant_state.to(device)
        return Params4bit(super().to(device=device, dtype=dtype, non_blocking=non_blocking),
                          requires_grad=self.requires_grad, quant_state=self.quant_state, blocksize=self.blocksize,
                          compress_statistics=self.compress_statistics, quant_type=self.quant_type,
                          quant_storage=self.quant_storage, bnb_quantized=self.bnb_quantized)


class Linear4bit(nn.Linear):
    """QLoRA-style 4-bit linear layer (ref:nn/modules.py:346-477)."""

    def __init__(self, input_features, output_features, bias=True, compute_dtype=None, compress_statistics=True,
                 quant_type="fp4", quant_storage=torch.uint8, device=None):
        super().__init__(input_features, output_features, bias, device)
        self.weight = Params4bit(self.weight.data, requires_grad=False, compress_statistics=compress_statistics,
                                 quant_type=quant_type, quant_storage=quant_storage, module=self)
        self.compute_dtype = compute_dtype
        self.compute_type_is_set = False
        self.quant_state = None
        self.quant_storage = quant_storage

    def set_compute_type(self, x):
        if x.dtype in [torch.float32, torch.bfloat16]:
            self.compute_dtype = x.dtype
        elif x.dtype == torch.float16:
            if self.compute_dtype == torch.float32 and (x.numel() == x.shape[-1]):
                warnings.warn("Input type into Linear4bit is torch.float16, but bnb_4bit_compute_dtype=torch.float32 "
                              "(default). This will lead to slow inference.")
                warnings.filterwarnings("ignore", message=".*inference.")
            if self.compute_dtype == torch.float32 and (x.numel() != x.shape[-1]):
                warnings.warn("Input type into Linear4bit is torch.float16, but bnb_4bit_compute_dtype=torch.float32 "
                              "(default). This will lead to slow inference or training speed.")
                warnings.filterwarnings("ignore", message=".*inference or training")

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        super()._save_to_state_dict(destination, prefix, keep_vars)
        if getattr(self.weight, "quant_state", None) is not None:
            for k, v in self.weight.quant_state.as_dict(packed=True).items():
                destination[prefix + "weight." + k] = v if keep_vars else v.detach()

    def forward(self, x: torch.Tensor):
        if self.bias is not None and self.bias.dtype != x.dtype:
            self.bias.data = self.bias.data.to(x.dtype)
        if getattr(self.weight, "quant_state", None) is None:
            if getattr(self, "quant_state", None) is not None:
                assert self.weight.shape[1] == 1
                if not isinstance(self.weight, Params4bit):
                    self.weight = Params4bit(self.weight, quant_storage=self.quant_storage, bnb_quantized=True)
                self.weight.quant_state = self.quant_state
            else:
                print("FP4 quantization state not initialized. Please call .cuda() or .to(device) on the LinearFP4 "
                      "layer first.")
        if not self.compute_type_is_set:
            self.set_compute_type(x)
            self.compute_type_is_set = True
        inp_dtype = x.dtype
        if self.compute_dtype is not None:
            x = x.to(self.compute_dtype)
        bias = None if self.bias is None else self.bias.to(self.compute_dtype)
        out = matmul_4bit(x, self.weight.t(), bias=bias, quant_state=self.weight.quant_state)
        return out.to(inp_dtype)


class LinearFP4(Linear4bit):
    def __init__(self, input_features, output_features, bias=True, compute_dtype=None, compress_statistics=True,
                 quant_storage=torch.uint8, device=None):
        super().__init__(input_features, output_features, bias, compute_dtype, compress_statistics, "fp4",
                         quant_storage, device)


class LinearNF4(Linear4bit):
    def __init__(self, input_features, output_features, bias=True, compute_dtype=None, compress_statistics=True,
                 quant_storage=torch.uint8, device=None):
        super().__init__(input_features, output_features, bias, compute_dtype, compress_statistics, "nf4",
                         quant_storage, device)


class Int8Params(torch.nn.Parameter):
    """Row-major int8 weight + per-row absmax (ref:nn/modules.py:559-632)."""

    def __new__(cls, data=None, requires_grad=True, has_fp16_weights=False, CB=None, SCB=None):
        if data is None:
            data = torch.empty(0)
        obj = torch.Tensor._make_subclass(cls, data, requires_grad)
        obj.CB = CB
        obj.SCB = SCB
        obj.has_fp16_weights = has_fp16_weights
        return obj

    def cuda(self, device=None):
        if self.has_fp16_weights:
            return super().cuda(device)
        B = self.data.contiguous().half().cuda(device)
        CB, CBt, SCB, SCBt, _ = F.double_quant(B)
        del CBt
        del SCBt
        self.data = CB
        self.CB = CB
        self.SCB = SCB
        return self

    def __deepcopy__(self, memo):
        return type(self).__new__(type(self), data=copy.deepcopy(self.data, memo), requires_grad=self.requires_grad,
                                  has_fp16_weights=self.has_fp16_weights, CB=copy.deepcopy(self.CB, memo),
                                  SCB=copy.deepcopy(self.SCB, memo))

    def to(self, *args, **kwargs):
        device, dtype, non_blocking, _ = torch._C._nn._parse_to(*args, **kwargs)
        if device is not None and device.type == "cuda" and self.data.device.type == "cpu":
            return self.cuda(device)
        new_param = Int8Params(super().to(device=device, dtype=dtype, non_blocking=non_blocking),
                               requires_grad=self.requires_grad, has_fp16_weights=self.has_fp16_weights)
        new_param.CB = self.CB
        new_param.SCB = self.SCB
        return new_param


def maybe_rearrange_weight(state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys, error_msgs):
    """Load-time un-tiling of turing/ampere int8 weights (ref:nn/modules.py:635-654)."""
    weight = state_dict.get(f"{prefix}weight")
    if weight is None:
        return
    weight_format = state_dict.pop(f"{prefix}weight_format", "row")
    if isinstance(weight_format, torch.Tensor):
        weight_format = weight_format.item()
    if isinstance(weight_format, int) and weight_format not in INVERSE_LINEAR_8BIT_WEIGHTS_FORMAT_MAPPING:
        raise ValueError(f"Expected supported weight format - got {weight_format}")
    elif isinstance(weight_format, int):
        weight_format = INVERSE_LINEAR_8BIT_WEIGHTS_FORMAT_MAPPING[weight_format]
    if weight_format != "row":
        raise NotImplementedError("tiled int8 checkpoints: load the row-major weight instead")


class Linear8bitLt(nn.Linear):
    """LLM.int8() linear layer (ref:nn/modules.py:657-821)."""

    def __init__(self, input_features: int, output_features: int, bias=True, has_fp16_weights=True,
                 memory_efficient_backward=False, threshold=0.0, index=None, device=None):
        super().__init__(input_features, output_features, bias, device)
        assert not memory_efficient_backward, ("memory_efficient_backward is no longer required and the argument is "
                                               "deprecated in 0.37.0 and will be removed in 0.39.0")
        self.state = MatmulLtState()
        self.index = index
        self.state.threshold = threshold
        self.state.has_fp16_weights = has_fp16_weights
        self.state.memory_efficient_backward = memory_efficient_backward
        if threshold > 0.0 and not has_fp16_weights:
            self.state.use_pool = True
        self.weight = Int8Params(self.weight.data, has_fp16_weights=has_fp16_weights, requires_grad=has_fp16_weights)
        self._register_load_state_dict_pre_hook(maybe_rearrange_weight)

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        super()._save_to_state_dict(destination, prefix, keep_vars)
        param_from_weight = getattr(self.weight, "SCB")
        param_from_state = getattr(self.state, "SCB")
        key_name, format_name = prefix + "SCB", prefix + "weight_format"
        if not self.state.has_fp16_weights:
            if param_from_weight is not None:
                destination[key_name] = param_from_weight if keep_vars else param_from_weight.detach()
                destination[format_name] = torch.tensor(0, dtype=torch.uint8)
            elif param_from_state is not None:
                destination[key_name] = param_from_state if keep_vars else param_from_state.detach()
                fmt = "row" if self.state.CxB is None else self.state.formatB
                destination[format_name] = torch.tensor(LINEAR_8BIT_WEIGHTS_FORMAT_MAPPING[fmt], dtype=torch.uint8)

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                                      error_msgs)
        for key in list(unexpected_keys):
            if key[len(prefix):] == "SCB":
                if self.weight.SCB is None:
                    raise RuntimeError("Loading a quantized checkpoint into non-quantized Linear8bitLt is not "
                                       "supported. Please call module.cuda() before module.load_state_dict()")
                self.weight.SCB.copy_(state_dict[key])
                if self.state.SCB is not None:
                    self.state.SCB = self.weight.SCB
                unexpected_keys.remove(key)

    def init_8bit_state(self):
        self.state.CB = self.weight.CB
        self.state.SCB = self.weight.SCB
        self.weight.CB = None
        self.weight.SCB = None

    def forward(self, x: torch.Tensor):
        self.state.is_training = self.training
        if self.weight.CB is not None:
            self.init_8bit_state()
        if self.bias is not None and self.bias.dtype != x.dtype:
            self.bias.data = self.bias.data.to(x.dtype)
        return matmul(x, self.weight, bias=self.bias, state=self.state)
