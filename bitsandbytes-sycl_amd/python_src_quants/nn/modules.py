"""4-bit and 8-bit linear layers on ROCm: the public surface of ref:python_src_quants/nn/modules.py:212-821.

Names, constructor arguments, attributes, state-dict keys and pickling behaviour follow the reference; the
implementation is this backend's own.  The layers hand their packed weights to `matmul_4bit` / `matmul`, which
run the gfx950 kernels (fused NF4/FP4 GEMM or GEMV, fused igemmlt + dequant)."""
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

# Attributes a Params4bit carries beside its data; pickled / copied as one record.
_PARAMS4BIT_FIELDS = ("blocksize", "compress_statistics", "quant_type", "quant_state", "quant_storage",
                      "bnb_quantized", "module")


class Params4bit(torch.nn.Parameter):
    """Packed 4-bit weight: holds the float weight until the first move to a GPU, which quantises it
    (ref:nn/modules.py:212-343).  After quantisation `data` is the uint8 [(N*K+1)//2, 1] storage and
    `quant_state` the matching QuantState."""

    def __new__(cls, data: Optional[torch.Tensor] = None, requires_grad=False, quant_state: Optional[QuantState] = None,
                blocksize: int = 64, compress_statistics: bool = True, quant_type: str = "fp4",
                quant_storage: torch.dtype = torch.uint8, module: Optional["Linear4bit"] = None,
                bnb_quantized: bool = False) -> "Params4bit":
        payload = torch.empty(0) if data is None else data
        param = torch.Tensor._make_subclass(cls, payload, requires_grad)
        param._set_fields(dict(blocksize=blocksize, compress_statistics=compress_statistics, quant_type=quant_type,
                               quant_state=quant_state, quant_storage=quant_storage, bnb_quantized=bnb_quantized,
                               module=module))
        param.data = payload
        return param

    def _set_fields(self, fields: Dict[str, Any]) -> None:
        for name in _PARAMS4BIT_FIELDS:
            setattr(self, name, fields[name])

    def _fields(self) -> Dict[str, Any]:
        return {name: getattr(self, name) for name in _PARAMS4BIT_FIELDS}

    # pickling: the record of fields plus the payload and its grad flag
    def __getstate__(self):
        record = self._fields()
        record.update(self.__dict__)
        record["data"], record["requires_grad"] = self.data, self.requires_grad
        return record

    def __setstate__(self, state):
        self._set_fields(state)
        self.data = state["data"]
        self.requires_grad = state["requires_grad"]

    def _replica(self, deep: bool, memo=None) -> "Params4bit":
        clone = type(self).__new__(type(self))
        record = self.__getstate__()
        if deep:
            record["quant_state"] = copy.deepcopy(record["quant_state"], memo)
            record["data"] = copy.deepcopy(record["data"], memo)
        clone.__setstate__(record)
        return clone

    def __deepcopy__(self, memo):
        return self._replica(True, memo)

    def __copy__(self):
        return self._replica(False)

    @classmethod
    def from_prequantized(cls, data: torch.Tensor, quantized_stats: Dict[str, Any], requires_grad: bool = False,
                          device="cuda", **kwargs) -> "Params4bit":
        """Wrap an already-packed weight and its serialised QuantState (ref:nn/modules.py:271-289): the path a
        saved Linear4bit / an NF4 checkpoint takes back onto the GPU without re-quantising."""
        state = QuantState.from_dict(qs_dict=quantized_stats, device=device)
        return cls(data.to(device), requires_grad=requires_grad, quant_state=state, blocksize=state.blocksize,
                   compress_statistics=state.nested, quant_type=state.quant_type, quant_storage=data.dtype,
                   module=None, bnb_quantized=True)

    def _quantize(self, device):
        packed, state = F.quantize_4bit(self.data.contiguous().to(device), blocksize=self.blocksize,
                                        compress_statistics=self.compress_statistics, quant_type=self.quant_type,
                                        quant_storage=self.quant_storage)
        self.data, self.quant_state, self.bnb_quantized = packed, state, True
        if self.module is not None:
            self.module.quant_state = state
        return self

    def cuda(self, device=None, non_blocking: bool = False):
        return self.to(device="cuda" if device is None else device, non_blocking=non_blocking)

    def to(self, *args, **kwargs):
        device, dtype, non_blocking, _ = torch._C._nn._parse_to(*args, **kwargs)
        if device is not None and device.type == "cuda" and not self.bnb_quantized:
            return self._quantize(device)
        if self.quant_state is not None:
            self.quant_state.to(device)
        moved = super().to(device=device, dtype=dtype, non_blocking=non_blocking)
        fields = self._fields()
        fields["module"] = None
        return Params4bit(moved, requires_grad=self.requires_grad, **fields)


class Linear4bit(nn.Linear):
    """QLoRA-style 4-bit linear layer (ref:nn/modules.py:346-477).  forward -> matmul_4bit: the GEMV kernel
    for one activation row without grad, otherwise the fused 4-bit GEMM."""

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
        """bf16/fp32 inputs set the compute dtype; fp16 into an fp32-configured layer only warns
        (ref:nn/modules.py:416-434)."""
        if x.dtype in (torch.float32, torch.bfloat16):
            self.compute_dtype = x.dtype
            return
        if x.dtype == torch.float16 and self.compute_dtype == torch.float32:
            single_row = x.numel() == x.shape[-1]
            tail = "inference." if single_row else "inference or training speed."
            warnings.warn("Input type into Linear4bit is torch.float16, but bnb_4bit_compute_dtype=torch.float32 "
                          f"(default). This will lead to slow {tail}")
            warnings.filterwarnings("ignore", message=".*inference." if single_row else ".*inference or training")

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        """Weight plus the packed QuantState entries `weight.<key>` (ref:nn/modules.py:436-445)."""
        super()._save_to_state_dict(destination, prefix, keep_vars)
        state = getattr(self.weight, "quant_state", None)
        if state is None:
            return
        for key, value in state.as_dict(packed=True).items():
            destination[f"{prefix}weight.{key}"] = value if keep_vars else value.detach()

    def _resolve_quant_state(self) -> Optional[QuantState]:
        state = getattr(self.weight, "quant_state", None)
        if state is not None:
            return state
        if getattr(self, "quant_state", None) is None:
            print("FP4 quantization state not initialized. Please call .cuda() or .to(device) on the LinearFP4 "
                  "layer first.")
            return None
        # the layer was given a packed weight and a state separately (e.g. by an FSDP-style wrapper)
        assert self.weight.shape[1] == 1
        if not isinstance(self.weight, Params4bit):
            self.weight = Params4bit(self.weight, quant_storage=self.quant_storage, bnb_quantized=True)
        self.weight.quant_state = self.quant_state
        return self.quant_state

    def forward(self, x: torch.Tensor):
        if self.bias is not None and self.bias.dtype != x.dtype:
            self.bias.data = self.bias.data.to(x.dtype)
        state = self._resolve_quant_state()
        if not self.compute_type_is_set:
            self.set_compute_type(x)
            self.compute_type_is_set = True
        in_dtype = x.dtype
        if self.compute_dtype is not None:
            x = x.to(self.compute_dtype)
        bias = None if self.bias is None else self.bias.to(self.compute_dtype)
        return matmul_4bit(x, self.weight.t(), bias=bias, quant_state=state).to(in_dtype)


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
    """Row-major int8 weight CB + per-row absmax SCB, produced by double_quant on the first move to a GPU
    (ref:nn/modules.py:559-632)."""

    def __new__(cls, data=None, requires_grad=True, has_fp16_weights=False, CB=None, SCB=None):
        payload = torch.empty(0) if data is None else data
        param = torch.Tensor._make_subclass(cls, payload, requires_grad)
        param.CB, param.SCB, param.has_fp16_weights = CB, SCB, has_fp16_weights
        return param

    def cuda(self, device=None):
        if self.has_fp16_weights:
            return super().cuda(device)
        half = self.data.contiguous().half().cuda(device)
        CB, _, SCB, _, _ = F.double_quant(half)   # only the row-normalised half is kept
        self.data, self.CB, self.SCB = CB, CB, SCB
        return self

    def __deepcopy__(self, memo):
        dup = lambda t: copy.deepcopy(t, memo)   # noqa: E731
        return type(self).__new__(type(self), data=dup(self.data), requires_grad=self.requires_grad,
                                  has_fp16_weights=self.has_fp16_weights, CB=dup(self.CB), SCB=dup(self.SCB))

    def to(self, *args, **kwargs):
        device, dtype, non_blocking, _ = torch._C._nn._parse_to(*args, **kwargs)
        if device is not None and device.type == "cuda" and self.data.device.type == "cpu":
            return self.cuda(device)
        moved = Int8Params(super().to(device=device, dtype=dtype, non_blocking=non_blocking),
                           requires_grad=self.requires_grad, has_fp16_weights=self.has_fp16_weights)
        moved.CB, moved.SCB = self.CB, self.SCB
        return moved


def untile_int8_weight(weight: torch.Tensor, weight_format: str, rows: int, cols: int) -> torch.Tensor:
    """A col32 / col_turing / col_ampere tiled int8 weight (padded shape, ref:functional.py:482-518) back to the
    row-major [rows, cols] matrix, with the HIP inverse-transform kernels (ctransform_{col32,turing,ampere}2row);
    replaces the reference's index-permutation undo_layout (ref:autograd/_functions.py:58-104).  The result
    lives on the GPU (the layer it is loaded into computes there)."""
    if weight_format == "row":
        return weight
    src = weight if weight.is_cuda else weight.to(torch.device("cuda", torch.cuda.current_device()))
    out, _ = F.transform(src.contiguous(), "row", state=((rows, cols), weight_format))
    return out


def maybe_rearrange_weight(state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys, error_msgs,
                           shape=None):
    """Load-time pre-hook (ref:nn/modules.py:635-654): reads and drops `weight_format` and un-tiles a tiled int8
    weight.  `shape` = the layer's (out_features, in_features), which crops the tile padding; without it the
    tiled tensor must hold whole tiles (as the reference requires)."""
    weight = state_dict.get(f"{prefix}weight")
    if weight is None:
        return
    weight_format = state_dict.pop(f"{prefix}weight_format", "row")
    if isinstance(weight_format, torch.Tensor):
        weight_format = weight_format.item()
    if isinstance(weight_format, int):
        if weight_format not in INVERSE_LINEAR_8BIT_WEIGHTS_FORMAT_MAPPING:
            raise ValueError(f"Expected supported weight format - got {weight_format}")
        weight_format = INVERSE_LINEAR_8BIT_WEIGHTS_FORMAT_MAPPING[weight_format]
    if weight_format != "row":
        rows, cols = shape if shape is not None else tuple(weight.shape)
        state_dict[f"{prefix}weight"] = untile_int8_weight(weight, weight_format, rows, cols)


class Linear8bitLt(nn.Linear):
    """LLM.int8() linear layer (ref:nn/modules.py:657-821): int8 weight rows (CB, SCB), the activation
    quantised per row at every forward, outlier columns above `threshold` kept in fp16."""

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
        self._register_load_state_dict_pre_hook(self._rearrange_hook)

    def _rearrange_hook(self, state_dict, prefix, *args):
        maybe_rearrange_weight(state_dict, prefix, *args, shape=(self.out_features, self.in_features))

    def _scb_and_format(self):
        """(SCB, weight-format code) to save, or None for an fp16-weight layer (ref:nn/modules.py:725-756).  This
        backend keeps CB row-major at every point, so the saved format is "row" unless a tiled CxB was given."""
        if self.state.has_fp16_weights:
            return None
        if self.weight.SCB is not None:
            return self.weight.SCB, LINEAR_8BIT_WEIGHTS_FORMAT_MAPPING["row"]
        if self.state.SCB is not None:
            fmt = "row" if self.state.CxB is None else self.state.formatB
            if fmt not in LINEAR_8BIT_WEIGHTS_FORMAT_MAPPING:
                raise ValueError(f"Unrecognized weights format {fmt}")
            return self.state.SCB, LINEAR_8BIT_WEIGHTS_FORMAT_MAPPING[fmt]
        return None

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        super()._save_to_state_dict(destination, prefix, keep_vars)
        saved = self._scb_and_format()
        if saved is not None:
            scb, fmt = saved
            destination[prefix + "SCB"] = scb if keep_vars else scb.detach()
            destination[prefix + "weight_format"] = torch.tensor(fmt, dtype=torch.uint8)

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                                      error_msgs)
        scb_key = prefix + "SCB"
        if scb_key not in unexpected_keys:
            return
        if self.weight.SCB is None:
            raise RuntimeError("Loading a quantized checkpoint into non-quantized Linear8bitLt is not supported. "
                               "Please call module.cuda() before module.load_state_dict()")
        self.weight.SCB.copy_(state_dict[scb_key])
        if self.state.SCB is not None:
            self.state.SCB = self.weight.SCB
        unexpected_keys.remove(scb_key)

    def init_8bit_state(self):
        """Move CB/SCB from the parameter into the matmul state on the first forward."""
        self.state.CB, self.state.SCB = self.weight.CB, self.weight.SCB
        self.weight.CB = self.weight.SCB = None

    def forward(self, x: torch.Tensor):
        self.state.is_training = self.training
        if self.weight.CB is not None:
            self.init_8bit_state()
        if self.bias is not None and self.bias.dtype != x.dtype:
            self.bias.data = self.bias.data.to(x.dtype)
        return matmul(x, self.weight, bias=self.bias, state=self.state)
