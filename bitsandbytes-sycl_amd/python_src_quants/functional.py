"""Functional surface of the quantized-matmul hot path, MI355X backend.

Mirrors ref:python_src_quants/functional.py for the hot-path functions (same names, argument
meaning, returned shapes/dtypes and error behaviour) with device type ``"cuda"`` (ROCm)
instead of ``"xpu"``.  Every GPU op crosses into the gfx950 C-ABI library through ctypes;
there is no CPU/torch fallback for them.
"""
from __future__ import annotations

import ctypes as ct
import functools
import os
import threading
import weakref
from functools import reduce
import operator
from typing import Any, Dict, Optional, Tuple

import torch
from torch import Tensor

from .cextension import lib
from .utils import pack_dict_to_tensor, unpack_tensor_to_dict

name2qmap: Dict[str, Tensor] = {}

dtype2bytes = {torch.float32: 4, torch.float16: 2, torch.bfloat16: 2, torch.uint8: 1, torch.int8: 1}

_BLOCKSIZES = [4096, 2048, 1024, 512, 256, 128, 64]


def prod(iterable):
    return reduce(operator.mul, iterable, 1)


# ----------------------------------------------------------------------------- quantisation maps
def create_linear_map(signed=True, total_bits=8, add_zero=True):
    """ref:functional.py:248-264"""
    sign = -1.0 if signed else 0.0
    total_values = 2**total_bits
    if add_zero or total_bits < 8:
        total_values = 2**total_bits if not signed else 2**total_bits - 1
    values = torch.linspace(sign, 1.0, total_values)
    gap = 256 - values.numel()
    if gap == 0:
        return values
    half = values.numel() // 2
    return torch.Tensor(values[:half].tolist() + [0] * gap + values[half:].tolist())


def create_normal_map(offset=0.9677083, use_extra_value=True):
    """ref:functional.py:267-294 (needs scipy)."""
    from scipy.stats import norm

    if use_extra_value:
        v1 = norm.ppf(torch.linspace(offset, 0.5, 9)[:-1]).tolist()
        v2 = [0] * (256 - 15)
        v3 = (-norm.ppf(torch.linspace(offset, 0.5, 8)[:-1])).tolist()
    else:
        v1 = norm.ppf(torch.linspace(offset, 0.5, 8)[:-1]).tolist()
        v2 = [0] * (256 - 14)
        v3 = (-norm.ppf(torch.linspace(offset, 0.5, 8)[:-1])).tolist()
    values = torch.Tensor(v1 + v2 + v3).sort().values
    values /= values.max()
    assert values.numel() == 256
    return values


def create_dynamic_map(signed=True, max_exponent_bits=7, total_bits=8):
    """Dynamic exponent/fraction 8-bit map, ref:functional.py:339-391."""
    data = []
    non_sign_bits = total_bits - 1
    additional_items = 2 ** (non_sign_bits - max_exponent_bits) - 1
    for i in range(max_exponent_bits):
        fraction_items = int(
            2 ** (i + non_sign_bits - max_exponent_bits) + 1
            if signed
            else 2 ** (i + non_sign_bits - max_exponent_bits + 1) + 1,
        )
        boundaries = torch.linspace(0.1, 1, fraction_items)
        means = (boundaries[:-1] + boundaries[1:]) / 2.0
        data += ((10 ** (-(max_exponent_bits - 1) + i)) * means).tolist()
        if signed:
            data += (-(10 ** (-(max_exponent_bits - 1) + i)) * means).tolist()
    if additional_items > 0:
        boundaries = torch.linspace(0.1, 1, additional_items + 1)
        means = (boundaries[:-1] + boundaries[1:]) / 2.0
        data += ((10 ** (-(max_exponent_bits - 1) + max_exponent_bits - 1)) * means).tolist()
        if signed:
            data += (-(10 ** (-(max_exponent_bits - 1) + max_exponent_bits - 1)) * means).tolist()
    data.append(0)
    data.append(1.0)
    assert len(data) == 2**total_bits
    data += [0] * (256 - len(data))
    data.sort()
    return Tensor(data)


def get_4bit_type(typename, device=None, blocksize=64):
    """16-entry 4-bit code tables, ref:functional.py:1020-1099."""
    if device is None:
        device = "cuda"
    if typename == "nf4":
        data = [-1.0, -0.6961928009986877, -0.5250730514526367, -0.39491748809814453,
                -0.28444138169288635, -0.18477343022823334, -0.09105003625154495, 0.0,
                0.07958029955625534, 0.16093020141124725, 0.24611230194568634, 0.33791524171829224,
                0.44070982933044434, 0.5626170039176941, 0.7229568362236023, 1.0]
    elif typename == "fp4":
        data = [0, 0.0625, 8.0, 12.0, 4.0, 6.0, 2.0, 3.0, -0, -0.0625, -8.0, -12.0, -4.0, -6.0, -2.0, -3.0]
    elif typename == "int4":
        data = [7, 6, 5, 4, 3, 2, 1, 0, -0, -1, -2, -3, -4, -5, -6, -7]
    elif typename == "af4":
        if blocksize != 64:
            raise NotImplementedError("4-bit AbnormalFloats currently only support blocksize 64.")
        data = [-1.0, -0.69441008, -0.51243739, -0.3736951, -0.25607552, -0.14982478, -0.04934812, 0.0,
                0.04273164, 0.12934483, 0.21961274, 0.31675666, 0.42563882, 0.55496234, 0.72424863, 1.0][::-1]
    else:
        raise NotImplementedError(f"Typename {typename} not supported")
    t = torch.tensor(data, device=device)
    t.div_(t.abs().max())
    assert t.numel() == 16
    return t


def _dynamic_map(device) -> Tensor:
    """The default dynamic map, cached once per device (the CPU copy is handed out as a clone
    because the CPU entry point rewrites code[0] in place, cpu_ops.cpp:20)."""
    if "dynamic" not in name2qmap:
        name2qmap["dynamic"] = create_dynamic_map()
    device = torch.device(device)
    if device.type == "cpu":
        return name2qmap["dynamic"].clone()
    key = f"dynamic@{device}"
    if key not in name2qmap:
        name2qmap[key] = name2qmap["dynamic"].to(device)
    return name2qmap[key]


def get_special_format_str():
    """Weight tile format for igemmlt (ref:functional.py:410-418 returns 'col_turing' on XPU)."""
    return "col_turing"


# ----------------------------------------------------------------------------- call plumbing
def is_on_gpu(tensors):
    """All non-None tensors on one GPU (ref:functional.py:425-458), else TypeError."""
    idx = None
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise TypeError(
                "All input tensors need to be on the same GPU, but found some tensors to not be on a GPU:\n "
                f"{[(t.shape, t.device) for t in tensors if t is not None]}",
            )
        d = t.get_device()
        if idx is None:
            idx = d
        elif d != idx:
            raise TypeError(
                "Input tensors need to be on the same GPU, but found the following tensor and device combinations:\n "
                f"{[(t.shape, t.device) for t in tensors if t is not None]}",
            )
    return True


def get_ptr(A: Optional[Tensor]) -> Optional[ct.c_void_p]:
    if A is None:
        return None
    return ct.c_void_p(A.data_ptr())


# Host cost per call matters on the decode path (a 4096 x 11008 GEMV runs ~9 us on the GPU): the
# device switch is skipped when the device is already current, and the library's (thread-local)
# stream is rebound only when torch's current stream changed (cached per Python thread).
_tls = threading.local()
_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _current_raw_stream(idx: int) -> int:
    if _raw_stream is not None:
        return _raw_stream(idx)
    return torch.cuda.current_stream(idx).cuda_stream


def _offset_on(state, device) -> Tensor:
    """The nested-statistics offset as a one-element fp32 tensor on `device` (only its pointer is passed)."""
    off = state.offset
    if torch.is_tensor(off) and off.is_cuda and off.dtype == torch.float32 and off.numel() == 1 and off.device == device:
        return off
    off = off if torch.is_tensor(off) else torch.tensor(float(off))
    return off.to(device=device, dtype=torch.float32).reshape(1)


_get_device = getattr(torch._C, "_cuda_getDevice", None) or torch.cuda.current_device


def pre_call(device):
    """Select the device (ref:functional.py:461-464) and bind the library to torch's current stream."""
    prev_device = _get_device()
    idx = device.index if isinstance(device, torch.device) else device
    if idx is None:
        idx = prev_device
    if idx != prev_device:
        torch.cuda.set_device(idx)
    stream = _current_raw_stream(idx)
    if getattr(_tls, "stream", None) != stream:
        lib.cset_stream(ct.c_void_p(stream))
        _tls.stream = stream
    return prev_device


def post_call(prev_device):
    if _get_device() != prev_device:
        torch.cuda.set_device(prev_device)
    err = lib.cget_last_error()
    if err:
        raise RuntimeError(f"bitsandbytes HIP kernel error: {lib.cget_last_error_message().decode()}")


# ----------------------------------------------------------------------------- QuantState
class QuantState:
    """Container for quantisation state components (ref:functional.py:625-798)."""

    valid_quant_types = ("fp4", "nf4")
    valid_qs_type_keys = [f"bitsandbytes__{x}" for x in valid_quant_types]
    valid_qs_keys = ["absmax", "quant_map", "nested_absmax", "nested_quant_map", "quant_state", "quant_type",
                     "blocksize", "dtype", "shape", "nested_blocksize", "nested_dtype", "nested_offset"]

    def __init__(self, absmax, shape=None, code=None, blocksize=None, quant_type=None, dtype=None, offset=None,
                 state2=None):
        self.absmax = absmax
        self.shape = shape
        self.code = code
        self.dtype = dtype
        self.blocksize = blocksize
        self.quant_type = quant_type
        self.offset = offset
        self.state2 = state2
        self.nested = state2 is not None

    def __get_item__(self, idx):
        if self.nested:
            list_repr = [self.absmax, self.shape, self.dtype, self.blocksize, [self.offset, self.state2], self.quant_type]
        else:
            list_repr = [self.absmax, self.shape, self.dtype, self.blocksize, None, self.quant_type]
        return list_repr[idx]

    @classmethod
    def from_dict(cls, qs_dict: Dict[str, Any], device: torch.device) -> "QuantState":
        qs_key = [k for k, v in qs_dict.items() if "quant_state" in k and isinstance(v, torch.Tensor)]
        if not len(qs_key) and "quant_type" not in qs_dict:
            raise ValueError("Expected packed or unpacked quant_state items, found neither")
        elif len(qs_key) != 1 or qs_key[0].split(".")[-1] not in cls.valid_qs_type_keys:
            raise ValueError(
                f"There should be exactly one `quant_state` item with ending from {cls.valid_qs_type_keys}.\n"
                f"Detected {qs_key}.",
            )
        if len(qs_key) == 1:
            qs_dict.update(unpack_tensor_to_dict(qs_dict.pop(qs_key[0])))
        qs_dict = {k.split(".")[-1]: v for k, v in qs_dict.items()}
        assert set(qs_dict.keys()).issubset(cls.valid_qs_keys)
        if "nested_absmax" in qs_dict:
            offset = torch.tensor(float(qs_dict["nested_offset"])).to(device)
            state2 = cls(absmax=qs_dict["nested_absmax"].to(device), blocksize=qs_dict["nested_blocksize"],
                         code=qs_dict["nested_quant_map"].to(device), dtype=getattr(torch, qs_dict["nested_dtype"]))
        else:
            offset, state2 = None, None
        return cls(quant_type=qs_dict["quant_type"], absmax=qs_dict["absmax"].to(device),
                   blocksize=qs_dict["blocksize"], code=qs_dict["quant_map"].to(device),
                   dtype=getattr(torch, qs_dict["dtype"]),
                   shape=torch.Size(qs_dict["shape"]) if qs_dict["shape"] is not None else None,
                   offset=offset, state2=state2)

    def as_dict(self, packed=False):
        qs_dict = {
            "quant_type": self.quant_type,
            "absmax": self.absmax,
            "blocksize": self.blocksize,
            "quant_map": self.code,
            "dtype": str(self.dtype).strip("torch."),
            "shape": tuple(self.shape),
        }
        if self.nested:
            qs_dict.update({
                "nested_absmax": self.state2.absmax,
                "nested_blocksize": self.state2.blocksize,
                "nested_quant_map": self.state2.code.clone(),
                "nested_dtype": str(self.state2.dtype).strip("torch."),
                "nested_offset": self.offset.item(),
            })
        if not packed:
            return qs_dict
        qs_packed = {k: v for k, v in qs_dict.items() if isinstance(v, torch.Tensor)}
        non_tensor = {k: v for k, v in qs_dict.items() if not isinstance(v, torch.Tensor)}
        qs_packed["quant_state." + "bitsandbytes__" + self.quant_type] = pack_dict_to_tensor(non_tensor)
        return qs_packed

    def to(self, device):
        self.absmax = self.absmax.to(device)
        if self.nested:
            self.offset = self.offset.to(device)
            self.state2.absmax = self.state2.absmax.to(device)
            self.state2.code = self.state2.code.to(device)

    def __eq__(self, other):
        if not isinstance(other, QuantState):
            return False
        return (
            torch.allclose(self.absmax, other.absmax, atol=1e-6)
            and self.shape == other.shape
            and torch.allclose(self.code, other.code, atol=1e-6)
            and self.dtype == other.dtype
            and self.blocksize == other.blocksize
            and self.quant_type == other.quant_type
            and (self.offset == other.offset if self.offset is not None and other.offset is not None
                 else self.offset is other.offset)
            and (self.state2 == other.state2 if self.state2 is not None and other.state2 is not None
                 else self.state2 is other.state2)
        )


# ----------------------------------------------------------------------------- 8-bit blockwise
_QB = {torch.float32: "fp32", torch.float16: "fp16", torch.bfloat16: "bf16"}


def quantize_blockwise(A: Tensor, code: Optional[Tensor] = None, absmax: Optional[Tensor] = None,
                       out: Optional[Tensor] = None, blocksize=4096, nested=False) -> Tuple[Tensor, QuantState]:
    """Blockwise dynamic 8-bit quantisation (ref:functional.py:801-918)."""
    if code is None:
        code = _dynamic_map(A.device)
    if absmax is None:
        n = A.numel()
        blocks = n // blocksize + (1 if n % blocksize > 0 else 0)
        absmax = torch.zeros((blocks,), device=A.device, dtype=torch.float32)
    if out is None:
        out = torch.zeros_like(A, dtype=torch.uint8)

    if A.device.type != "cpu":
        assert blocksize in _BLOCKSIZES
        prev_device = pre_call(A.device)
        code = code.to(A.device)
        is_on_gpu([code, A, out, absmax])
        if A.dtype not in _QB:
            raise ValueError(f"Blockwise quantization only supports 16/32-bit floats, but got {A.dtype}")
        fn = getattr(lib, f"cquantize_blockwise_{_QB[A.dtype]}")
        fn(get_ptr(code), get_ptr(A), get_ptr(absmax), get_ptr(out), ct.c_int32(blocksize), ct.c_int(A.numel()))
        post_call(prev_device)
    else:
        # host tensors: the reference's CPU entry point (ref:functional.py:885-895), run on the host cores by
        # the library (cpu_ops.cpp; no GPU needed).  It takes fp32 only: other dtypes are converted first
        # (the reference passes their pointer unchanged and the C side misreads them).
        code = code.cpu()
        A32 = A if (A.dtype == torch.float32 and A.is_contiguous()) else A.float().contiguous()
        lib.cquantize_blockwise_cpu_fp32(get_ptr(code), get_ptr(A32), get_ptr(absmax), get_ptr(out),
                                         ct.c_longlong(blocksize), ct.c_longlong(A.numel()))

    if nested:
        offset = absmax.mean()
        absmax -= offset
        qabsmax, state2 = quantize_blockwise(absmax, blocksize=blocksize, nested=False)
        quant_state = QuantState(absmax=qabsmax, code=code, blocksize=blocksize, dtype=A.dtype, offset=offset,
                                 state2=state2)
    else:
        quant_state = QuantState(absmax=absmax, code=code, blocksize=blocksize, dtype=A.dtype)
    return out, quant_state


def dequantize_blockwise(A: Tensor, quant_state: Optional[QuantState] = None, absmax: Optional[Tensor] = None,
                         code: Optional[Tensor] = None, out: Optional[Tensor] = None, blocksize: int = 4096,
                         nested=False) -> Tensor:
    """ref:functional.py:921-1017"""
    assert quant_state is not None or absmax is not None
    if code is None and quant_state is None:
        code = _dynamic_map(A.device)
    if quant_state is None:
        quant_state = QuantState(absmax=absmax, code=code, blocksize=blocksize, dtype=torch.float32)

    absmax = quant_state.absmax
    if quant_state.nested:
        absmax = dequantize_blockwise(quant_state.absmax, quant_state.state2)
        absmax += quant_state.offset
        if absmax.dtype != torch.float32:
            absmax = absmax.float()

    if out is None:
        out = torch.empty(A.shape, dtype=quant_state.dtype, device=A.device)

    if A.device.type != "cpu":
        prev_device = pre_call(A.device)
        code = quant_state.code.to(A.device)
        if quant_state.blocksize not in [2048, 4096, 1024, 512, 256, 128, 64]:
            raise ValueError(
                f"The blockwise of {quant_state.blocksize} is not supported. "
                "Supported values: [2048, 4096, 1024, 512, 256, 128, 64]",
            )
        is_on_gpu([A, absmax, out])
        if out.dtype not in _QB:
            raise ValueError(f"Blockwise quantization only supports 16/32-bit floats, but got {A.dtype}")
        fn = getattr(lib, f"cdequantize_blockwise_{_QB[out.dtype]}")
        fn(get_ptr(code), get_ptr(A), get_ptr(absmax), get_ptr(out), ct.c_int(quant_state.blocksize),
           ct.c_int(A.numel()))
        post_call(prev_device)
    else:
        # host tensors (ref:functional.py:1006-1015), run on the host cores.  The decoded fp32 absmax is passed
        # (the reference passes quant_state.absmax, i.e. the uint8 codes, when the statistics are nested).
        code = quant_state.code.cpu()
        absmax = absmax.float().contiguous()
        o32 = out if (out.dtype == torch.float32 and out.is_contiguous()) else torch.empty(A.shape, dtype=torch.float32)
        Ac = A.contiguous()   # bound to a name: the C call must not see a freed temporary
        lib.cdequantize_blockwise_cpu_fp32(get_ptr(code), get_ptr(Ac), get_ptr(absmax), get_ptr(o32),
                                           ct.c_longlong(quant_state.blocksize), ct.c_longlong(A.numel()))
        if o32 is not out:
            out.copy_(o32)
    return out


# ----------------------------------------------------------------------------- 4-bit
def quantize_fp4(A, absmax=None, out=None, blocksize=64, compress_statistics=False, quant_storage=torch.uint8):
    return quantize_4bit(A, absmax, out, blocksize, compress_statistics, "fp4", quant_storage)


def quantize_nf4(A, absmax=None, out=None, blocksize=64, compress_statistics=False, quant_storage=torch.uint8):
    return quantize_4bit(A, absmax, out, blocksize, compress_statistics, "nf4", quant_storage)


def quantize_4bit(A: Tensor, absmax: Optional[Tensor] = None, out: Optional[Tensor] = None, blocksize=64,
                  compress_statistics=False, quant_type="fp4",
                  quant_storage=torch.uint8) -> Tuple[Tensor, QuantState]:
    """Blockwise FP4/NF4 quantisation (ref:functional.py:1124-1268)."""
    if A.device.type != "cuda":
        raise NotImplementedError(f"Device type not supported for FP4 quantization: {A.device.type}")
    if quant_type not in ["fp4", "nf4"]:
        raise NotImplementedError(f"4-bit quantization data type {quant_type} is not implemented.")
    n = A.numel()
    input_shape = A.shape
    if absmax is None:
        blocks = n // blocksize + (1 if n % blocksize > 0 else 0)
        absmax = torch.zeros((blocks,), device=A.device, dtype=torch.float32)
    if out is None:
        mod = dtype2bytes[quant_storage] * 2
        out = torch.zeros(((n + 1) // mod, 1), dtype=quant_storage, device=A.device)
    assert blocksize in _BLOCKSIZES

    prev_device = pre_call(A.device)
    is_on_gpu([A, out, absmax])
    if A.dtype not in _QB:
        raise ValueError(f"Blockwise quantization only supports 16/32-bit floats, but got {A.dtype}")
    fn = getattr(lib, f"cquantize_blockwise_{_QB[A.dtype]}_{quant_type}")
    fn(get_ptr(None), get_ptr(A), get_ptr(absmax), get_ptr(out), ct.c_int32(blocksize), ct.c_int(n))
    post_call(prev_device)

    code = get_4bit_type(quant_type, device=A.device)
    if compress_statistics:
        offset = absmax.mean()
        absmax -= offset
        qabsmax, state2 = quantize_blockwise(absmax, blocksize=256)
        del absmax
        state = QuantState(absmax=qabsmax, shape=input_shape, dtype=A.dtype, blocksize=blocksize, code=code,
                           quant_type=quant_type, offset=offset, state2=state2)
    else:
        state = QuantState(absmax=absmax, shape=input_shape, dtype=A.dtype, blocksize=blocksize, code=code,
                           quant_type=quant_type)
    return out, state


def dequantize_fp4(A, quant_state=None, absmax=None, out=None, blocksize: int = 64):
    return dequantize_4bit(A, quant_state, absmax, out, blocksize, "fp4")


def dequantize_nf4(A, quant_state=None, absmax=None, out=None, blocksize: int = 64):
    return dequantize_4bit(A, quant_state, absmax, out, blocksize, "nf4")


def _nested_stats_in_kernel_ok(state: QuantState) -> bool:
    """Compressed statistics a kernel can decode in place: contiguous uint8 codes, a contiguous fp32 second level
    and a contiguous fp32 256-entry map, a power-of-two nested blocksize (what the in-kernel decoders read)."""
    if not state.nested or state.absmax.dtype != torch.uint8 or not state.absmax.is_contiguous():
        return False
    s2 = state.state2
    bs2 = s2.blocksize
    return (s2.absmax.dtype == torch.float32 and s2.absmax.is_contiguous() and s2.code is not None
            and s2.code.dtype == torch.float32 and s2.code.is_contiguous() and s2.code.numel() >= 256
            and bs2 > 0 and (bs2 & (bs2 - 1)) == 0)


def _absmax_fp32(state: QuantState) -> Tensor:
    """Per-block fp32 absmax, resolving nested statistics (ref:functional.py:1346-1350, 1982-1984)."""
    absmax = state.absmax
    if state.nested:
        s2 = state.state2
        bs2 = s2.blocksize
        off = state.offset if isinstance(state.offset, torch.Tensor) else None
        if (absmax.is_cuda and absmax.dtype == torch.uint8 and absmax.is_contiguous() and s2.absmax.dtype == torch.float32
                and s2.code is not None and s2.code.is_cuda and off is not None and off.is_cuda
                and off.dtype == torch.float32 and bs2 > 0 and (bs2 & (bs2 - 1)) == 0):
            # one launch: code2[q] * absmax2 + offset (the two fp32 roundings of the two-step path)
            out = torch.empty(absmax.numel(), dtype=torch.float32, device=absmax.device)
            prev_device = pre_call(absmax.device)
            lib.cdequantize_nested_absmax_fp32(get_ptr(s2.code), get_ptr(absmax), get_ptr(s2.absmax), get_ptr(off),
                                               get_ptr(out), ct.c_int32(bs2), ct.c_longlong(absmax.numel()))
            post_call(prev_device)
            return out.view(absmax.shape)
        absmax = dequantize_blockwise(state.absmax, state.state2)
        absmax += state.offset
        if absmax.dtype != torch.float32:
            absmax = absmax.float()
    return absmax


def _dequant_4bit_nested(A: Tensor, state: QuantState, out: Tensor) -> bool:
    """One launch: the 4-bit dequantise with the compressed statistics decoded in the kernel
    (cdequantize_blockwise_nested_*).  False when the dtype/shape needs the two-step path."""
    if out.dtype not in (torch.float16, torch.bfloat16) or not _nested_stats_in_kernel_ok(state):
        return False
    s2 = state.state2
    offset = _offset_on(state, A.device)
    prev_device = pre_call(A.device)
    is_on_gpu([A, state.absmax, s2.code, s2.absmax, offset, out])
    qt = "fp4" if state.quant_type == "fp4" else "nf4"
    fn = getattr(lib, f"cdequantize_blockwise_nested_{_QB[out.dtype]}_{qt}")
    rc = fn(get_ptr(A), get_ptr(state.absmax), get_ptr(s2.code), get_ptr(s2.absmax), get_ptr(offset), get_ptr(out),
            ct.c_int32(state.blocksize), ct.c_int32(s2.blocksize), ct.c_longlong(out.numel()))
    post_call(prev_device)
    return rc == 0


def dequantize_4bit(A: Tensor, quant_state: Optional[QuantState] = None, absmax: Optional[Tensor] = None,
                    out: Optional[Tensor] = None, blocksize: int = 64, quant_type="fp4") -> Tensor:
    """ref:functional.py:1291-1424"""
    if blocksize not in [2048, 4096, 1024, 512, 256, 128, 64]:
        raise ValueError(
            f"The blockwise of {blocksize} is not supported. Supported values: [2048, 4096, 1024, 512, 256, 128, 64]",
        )
    if quant_type not in ["fp4", "nf4"]:
        raise NotImplementedError(f"4-bit quantization data type {quant_type} is not implemented.")
    if quant_state is None:
        assert absmax is not None and out is not None
        quant_state = QuantState(absmax=absmax, shape=out.shape, dtype=out.dtype, blocksize=blocksize,
                                 quant_type=quant_type)
    else:
        absmax = quant_state.absmax
    if out is None:
        out = torch.empty(quant_state.shape, dtype=quant_state.dtype, device=A.device)
    n = out.numel()
    if quant_state.nested and _dequant_4bit_nested(A, quant_state, out):
        if A.shape[0] == 1:   # is_transposed (ref:functional.py:1420-1424)
            return out.t()
        return out
    if quant_state.nested:
        absmax = _absmax_fp32(quant_state)

    prev_device = pre_call(A.device)
    is_on_gpu([A, absmax, out])
    if out.dtype not in _QB:
        raise ValueError(f"Blockwise quantization only supports 16/32-bit floats, but got {A.dtype}")
    qt = "fp4" if quant_state.quant_type == "fp4" else "nf4"
    fn = getattr(lib, f"cdequantize_blockwise_{_QB[out.dtype]}_{qt}")
    fn(get_ptr(None), get_ptr(A), get_ptr(absmax), get_ptr(out), ct.c_int(quant_state.blocksize), ct.c_int(n))
    post_call(prev_device)

    if A.shape[0] == 1:   # is_transposed (ref:functional.py:1420-1424)
        return out.t()
    return out


# ----------------------------------------------------------------------------- 4-bit matmul
class _GemvPlan:
    """The per-weight part of a decode GEMV call, prepared once: the entry point (with ctypes argtypes, so
    plain ints pass without wrapper objects), the statistics pointers and the integer arguments.  It holds
    the statistics tensors it points at and is used only while the state still holds the same objects."""
    __slots__ = ("fn", "nested", "absmax", "code", "s2", "s2absmax", "s2code", "offset_src", "offset", "dev", "m",
                 "head", "mid", "tail")

    def valid(self, state, dev) -> bool:
        if self.dev != dev or self.absmax is not state.absmax or self.code is not state.code:
            return False
        if not self.nested:
            return state.state2 is None
        s2 = state.state2
        return (s2 is self.s2 and s2.absmax is self.s2absmax and s2.code is self.s2code
                and state.offset is self.offset_src)


# id(state) -> (weak reference to the state, {(dtype, device): plan}); the entry leaves with the state
# (QuantState defines __eq__ and so is unhashable: keyed by id, checked by identity)
_GEMV_PLANS: Dict[int, Tuple[Any, Dict]] = {}
_I32, _PTR = ct.c_int32, ct.c_void_p


def _gemv_plan(A: Tensor, state) -> Optional[_GemvPlan]:
    """Build (or fetch) the cached plan for a bf16/fp16 decode GEMV against `state`; None when the call
    needs the general path (fp32 activations, an fp32 absmax that must be decoded first)."""
    names = {torch.float16: "fp16", torch.bfloat16: "bf16"}
    if A.dtype not in names:
        return None
    dev = A.get_device()
    entry = _GEMV_PLANS.get(id(state))
    per_state = entry[1] if entry is not None and entry[0]() is state else None
    key = (A.dtype, dev)
    if per_state is not None:
        plan = per_state.get(key)
        if plan is not None and plan.valid(state, dev):
            return plan
    m, k = state.shape[0], state.shape[1]
    plan = _GemvPlan()
    plan.dev, plan.m, plan.absmax, plan.code = dev, m, state.absmax, state.code
    plan.nested = A.dtype != torch.float32 and _nested_stats_in_kernel_ok(state)
    ldb, ldm = (k + 1) // 2, m
    if plan.nested:
        s2 = state.state2
        plan.s2, plan.s2absmax, plan.s2code = s2, s2.absmax, s2.code
        plan.offset_src, plan.offset = state.offset, _offset_on(state, A.device)
        is_on_gpu([state.absmax, s2.absmax, s2.code, plan.offset, state.code])
        plan.fn = getattr(lib, f"cgemm_4bit_inference_naive_nested_{names[A.dtype]}")
        plan.fn.argtypes = [_I32] * 3 + [_PTR] * 8 + [_I32] * 5
        plan.head = (m, 1, k)
        plan.mid = (state.absmax.data_ptr(), s2.code.data_ptr(), s2.absmax.data_ptr(), plan.offset.data_ptr(),
                    state.code.data_ptr())
        plan.tail = (ldm, ldb, ldm, state.blocksize, s2.blocksize)
    else:
        if state.state2 is not None or state.absmax.dtype != torch.float32:
            return None                      # compressed statistics the kernel cannot decode: general path
        plan.s2 = plan.s2absmax = plan.s2code = plan.offset_src = plan.offset = None
        is_on_gpu([state.absmax, state.code])
        plan.fn = getattr(lib, f"cgemm_4bit_inference_naive_{names[A.dtype]}")
        plan.fn.argtypes = [_I32] * 3 + [_PTR] * 5 + [_I32] * 4
        plan.head = (m, 1, k)
        plan.mid = (state.absmax.data_ptr(), state.code.data_ptr())
        plan.tail = (ldm, ldb, ldm, state.blocksize)
    if per_state is None:
        sid = id(state)
        per_state = {}
        _GEMV_PLANS[sid] = (weakref.ref(state, lambda _r, sid=sid: _GEMV_PLANS.pop(sid, None)), per_state)
    per_state[key] = plan
    return plan


def _gemv_out(A: Tensor, bout: int) -> Tensor:
    if len(A.shape) == 3:
        return torch.empty(size=(A.shape[0], A.shape[1], bout), dtype=A.dtype, device=A.device)
    return torch.empty(size=(A.shape[0], bout), dtype=A.dtype, device=A.device)


def gemv_4bit(A: Tensor, B: Tensor, out: Optional[Tensor] = None, transposed_A=False, transposed_B=False,
              state=None):
    """4-bit GEMV for a single activation row (ref:functional.py:1961-2060).

    bf16/fp16 calls against the same weight reuse a prepared plan (_gemv_plan), so the host cost per call is
    the checks below, the output allocation, the stream binding and one ctypes call."""
    if state is None:
        raise ValueError("state cannot None. gem_4bit( ) requires the state from quantize_4bit( )")
    if A.numel() != A.shape[-1]:
        raise ValueError(
            'Dimensions of A are invalid. Must be a vector with the leading dimensions of "1", e.g. [1, 1, 2048]',
        )
    if B.dtype not in (torch.uint8, torch.bfloat16, torch.float16, torch.float32):
        raise NotImplementedError(f"Matmul not implemented for data type {A.dtype}")
    plan = _gemv_plan(A, state) if A.is_cuda else None
    if plan is not None and B.is_cuda and B.get_device() == plan.dev:
        if out is None:
            out = _gemv_out(A, plan.m)
        elif not out.is_cuda or out.get_device() != plan.dev:
            is_on_gpu([A, out])
        prev_device = pre_call(A.device)
        rc = plan.fn(*plan.head, A.data_ptr(), B.data_ptr(), *plan.mid, out.data_ptr(), *plan.tail)
        if plan.nested and rc == 0:          # launched, no error recorded (2 = launch error, 1 = declined)
            if prev_device != plan.dev:
                torch.cuda.set_device(prev_device)
            return out
        if rc != 1 or not plan.nested:
            post_call(prev_device)
            return out
        torch.cuda.set_device(prev_device)   # nested shape the kernel declined: general path below
    prev_device = pre_call(A.device)
    Bshape = state.shape
    bout = Bshape[0]
    if out is None:
        out = _gemv_out(A, bout)
    m, n, k = Bshape[0], 1, Bshape[1]
    lda, ldc, ldb = Bshape[0], Bshape[0], (A.shape[-1] + 1) // 2
    names = {torch.float16: "fp16", torch.bfloat16: "bf16", torch.float32: "fp32"}
    if A.dtype not in names:
        raise NotImplementedError(f"Matmul not implemented for data type {A.dtype}")
    absmax = _absmax_fp32(state)
    is_on_gpu([B, A, out, absmax, state.code])
    fn = getattr(lib, f"cgemm_4bit_inference_naive_{names[A.dtype]}")
    fn(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k), get_ptr(A), get_ptr(B), get_ptr(absmax), get_ptr(state.code),
       get_ptr(out), ct.c_int32(lda), ct.c_int32(ldb), ct.c_int32(ldc), ct.c_int32(state.blocksize))
    post_call(prev_device)
    return out


def gemm_4bit_supported(A: Tensor, state: QuantState) -> bool:
    return (A.dtype in (torch.bfloat16, torch.float16) and A.is_cuda and state.shape[1] % 64 == 0
            and A.shape[-1] == state.shape[1] and state.blocksize >= 64)


_GEMM_WS: dict = {}


def _stream_key(device):
    idx = device.index if isinstance(device, torch.device) else device
    return _current_raw_stream(torch.cuda.current_device() if idx is None else idx)


def _gemm_workspace(device, nbytes: int) -> Optional[Tensor]:
    """Grow-only fp32 split-K workspace per (device, stream) for gemm_4bit (cgemm_4bit_workspace_bytes);
    kept across calls so steady-state calls (and HIP-graph replays) allocate nothing, and never shared
    by two streams that could run GEMMs concurrently."""
    if nbytes <= 0:
        return None
    key = (device, _stream_key(device))
    ws = _GEMM_WS.get(key)
    if ws is None or ws.numel() * 4 < nbytes:
        ws = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=device)
        _GEMM_WS[key] = ws
    return ws


# Prefill routing (gemm_4bit_static_route, round 4): from GEMM_4BIT_DEQUANT_MIN_ROWS activation rows always the
# reference's own M > 1 algorithm -- dequantise the whole weight (the HIP kernel, HBM-bound) and one bf16/fp16 GEMM,
# here the hand-written k_hgemm; below that the same pair except on deep, wide weights with few rows, where the
# one-kernel fused NF4 GEMM wins (see the route's docstring).  GEMM_4BIT_DEQUANT_MIN_FEATURES: kept for callers and
# tests that size a "large prefill" problem (the static rule no longer needs it).
GEMM_4BIT_DEQUANT_MIN_ROWS = 2048
GEMM_4BIT_DEQUANT_MIN_FEATURES = 1024
# Up to this many activation rows the C side runs the few-token kernels (gemm4bit_fewtok.hip whole-K up to 32 rows,
# gemm4bit_skinny.hip split-K at 33..64 rows; round 2: 11008 x 4096 at 33..64 rows 43.7 -> 27.3..31.2 us against the
# library pair, profiles/lab/r02_fewtoken_64rows.txt); with nested statistics the Python side calls its one-launch
# entry point directly.
GEMM_4BIT_FEW_TOKENS = 64
# (round 2's rule for 65..256 rows of wide weights; the round-4 static rule covers those rows with k_hgemm's 128-row
# tile and split-K -- 11008 x 4096 at 96 / 128 / 256 rows 52.5 / 54.0 / 60.4 us against the library pair's 48.9 / 51.8
# / 58.7 and the fused kernel's 62.1 / 66.2 / 74.0, profiles/lab/r04_route_sweep.txt)
GEMM_4BIT_WIDE_MAX_ROWS = 256
# 2..GEMM_4BIT_GEMV_TOKENS activation rows: where the C side's rule takes the shape (cgemm_4bit_fewtok_takes; round 3,
# measured faster), the whole-K MFMA few-token kernel (gemm4bit_fewtok.hip); elsewhere the multi-row GEMV
# (gemv4bit_tok.hip: every weight byte looked up once and dotted with each row, whole K per workgroup, one launch,
# rows bit-identical to gemv_4bit on each row).  Batch invariance is therefore given up by default: on the MFMA kernel
# a row of a 2..4-row batch is within the GEMV tolerance of gemv_4bit on that row, not bit-identical to it (both are
# deterministic run to run; tests/test_matmul4bit_gpu.py::test_fewtok_default_rows_close_to_gemv_and_deterministic).
# set_fewtok_mode(1) restores the bit-identical multi-row GEMV.
GEMM_4BIT_GEMV_TOKENS = 4

# The GEMM after the dequantise is the hand-written k_hgemm (hgemm.hip, chgemm_tn_*: 4 waves on v_mfma_f32_16x16x32,
# 256 x 256 tiles -- 128 x 128 per wave -- or the half-width 256 x 128 / 128 x 256 tiles, split-K over the GEMM
# workspace on small grids; the C side's launch plan, hgemm.hip hgemm_plan / chgemm_tn_plan) on every shape it takes
# (_hgemm_fits).  HGEMM_MIN_TILES: the 256 x 256 grid size from which no split is considered.
HGEMM_MIN_TILES = 192

# Routing is deterministic by default: the static rule above picks the kernel from the shape alone, so every process
# and every rank runs the same kernels on the same shape and returns the same bits.  BNB_ROUTE_TUNING=1 (or
# GEMM_4BIT_ROUTE_TUNING = True) measures instead: the first call of a prefill shape (more than GEMM_4BIT_FEW_TOKENS
# rows; per device, dtype and statistics format) times "hgemm" (dequantise + k_hgemm), "library" (dequantise +
# torch.matmul), "library_tn" (dequantise + cgemm_tn_*, rocBLAS with the per-shape solution search of gemm_lib.hip)
# and "fused" (the one-kernel NF4 GEMM) on its own operands (one warm call each, then the best of three interleaved
# rounds) and leaves the static rule's route only for one faster by more than GEMM_4BIT_ROUTE_MARGIN; nothing is timed
# during HIP-graph capture.  Choices are cached per quarter-octave bucket of the row count (_route_rows_bucket) and,
# with BNB_ROUTE_PLAN=<file>, persisted as JSON and read back by later processes (and by every rank of a job that
# shares the file), so a measured route is reproducible across processes too.  export_routes() / import_routes()
# hand the table over explicitly (e.g. broadcast from rank 0).
GEMM_4BIT_ROUTE_TUNING = os.environ.get("BNB_ROUTE_TUNING", "0") == "1"
GEMM_4BIT_ROUTE_MARGIN = 0.05
GEMM_4BIT_ROUTES = ("hgemm", "library", "library_tn", "fused")
_ROUTES: dict = {}
_ROUTE_PLAN_LOADED = [False]

_DEQ_WS: dict = {}
_DEQ_META: dict = {}


def _route_rows_bucket(rows: int) -> int:
    """Row counts share a measured route within quarter-octave buckets (4096..5119 -> 4096, 5120..6143 -> 5120, ...),
    so variable-length prefill measures at most four buckets per octave and weight shape, not every length."""
    step = 1 << max(0, rows.bit_length() - 3)
    return rows // step * step


@functools.lru_cache(maxsize=None)
def _device_name(index: int) -> str:
    try:
        return torch.cuda.get_device_name(index)
    except Exception:  # noqa: BLE001
        return "unknown"


def _route_key(A2: Tensor, state: QuantState, absmax: Optional[Tensor]):
    # the device's NAME (not its index): a plan file measured on one MI355X applies to every MI355X of the job
    return (_device_name(A2.device.index), _route_rows_bucket(A2.shape[0]), state.shape[0], state.shape[1],
            str(A2.dtype), state.quant_type, state.blocksize, bool(state.nested and absmax is None))


def _plan_path() -> Optional[str]:
    return os.environ.get("BNB_ROUTE_PLAN") or None


def _load_route_plan():
    if _ROUTE_PLAN_LOADED[0]:
        return
    _ROUTE_PLAN_LOADED[0] = True
    path = _plan_path()
    if path and os.path.exists(path):
        import json
        with open(path) as f:
            import_routes(json.load(f))


def _save_route_plan():
    """Merge this process's measured routes into the plan file: under an exclusive lock on `<plan>.lock`, re-read the
    file, add the entries it does not hold yet (a route another rank measured first wins, so every process that reads
    the file afterwards routes the same way), adopt its entries here too, and replace it atomically.  A plan that
    cannot be written (missing directory, permissions) is a warning, never an error of the GEMM call."""
    path = _plan_path()
    if not path:
        return
    import fcntl
    import json
    import tempfile
    import warnings
    try:
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        with open(path + ".lock", "a") as lk:
            fcntl.flock(lk, fcntl.LOCK_EX)
            try:
                if os.path.exists(path):
                    with open(path) as f:
                        on_disk = json.load(f)
                    for row in on_disk.get("routes", []):
                        *key, route = row
                        if route in GEMM_4BIT_ROUTES and len(key) == 8:
                            _ROUTES[tuple(key)] = route     # the first measurement on disk wins
                fd, tmp = tempfile.mkstemp(dir=d, prefix=".route_plan")
                with os.fdopen(fd, "w") as f:
                    json.dump(export_routes(), f, indent=1)
                os.replace(tmp, path)   # atomic: a concurrent reader sees the old or the new table, never half of one
            finally:
                fcntl.flock(lk, fcntl.LOCK_UN)
    except (OSError, ValueError) as ex:
        warnings.warn(f"gemm_4bit route plan {path!r} not written: {ex}")


def export_routes() -> dict:
    """The measured route table as JSON-able data: {"version": 1, "routes": [[key..., route], ...]}."""
    return {"version": 1, "routes": [list(k) + [r] for k, r in sorted(_ROUTES.items(), key=lambda kv: str(kv[0]))]}


def import_routes(table: dict) -> int:
    """Merge a table from export_routes() (entries naming an unknown route are ignored); returns the entry count."""
    n = 0
    for row in table.get("routes", []):
        *key, route = row
        if route in GEMM_4BIT_ROUTES and len(key) == 8:
            _ROUTES[tuple(key)] = route
            n += 1
    return n


def gemm_4bit_measured_route(A: Tensor, state: QuantState, absmax: Optional[Tensor] = None) -> Optional[str]:
    """The measured route cached for A's rows against this weight, or None when the shape has not been measured (the
    static rule applies)."""
    _load_route_plan()
    return _ROUTES.get(_route_key(A.reshape(-1, state.shape[1]), state, absmax))


def _hgemm_fits(rows: int, N: int, K: int) -> bool:
    """chgemm_tn's own rule: k % 64 == 0 and every 32-bit lane offset (row * K * 2 bytes) below 4 GiB.  Round 4: the
    hand-written GEMM is the static choice wherever it fits -- full grids unsplit, grids below 192 tiles of 256 x 256
    as split-K over the GEMM workspace (chgemm_tn_ws_*; N % 4 == 0, else unsplit); the library GEMM only where this
    rule fails.  Round-3 measurements (tools/route_probe3.py, profiles/lab/r03_routes.txt): 4096 x 1024 x 28672 (the
    70B down-projection shard) 207 us split-K against 342 (torch.matmul) and 228 (rocBLAS searched); 4096 x 1024 x 8192
    76.7 vs 74.8 us on torch.matmul."""
    return (K % 64 == 0 and rows >= 1 and N >= 1
            and (rows - 1) * K * 2 + 2 * K <= 0xFFFFFFFF and (N - 1) * K * 2 + 2 * K <= 0xFFFFFFFF)


_U32 = 0xFFFFFFFF


def _hgemm_chunks(rows: int, N: int, K: int, blocksize: int) -> Tuple[int, int]:
    """(row chunk, weight-row chunk) sizes for a product k_hgemm cannot take in one launch (_hgemm_fits: 32-bit lane
    offsets).  Row chunks: the most activation rows whose offsets fit, rounded down to whole 256-row tiles.  Weight
    chunks: the most weight rows whose bf16 copy fits the same bound and the dequantise's 32-bit element count, a
    multiple of 256 rows and of whole statistics blocks (so every chunk starts on a block boundary)."""
    rc = rows if (rows - 1) * K * 2 + 2 * K <= _U32 else max(256, ((_U32 - 2 * K) // (2 * K) + 1) // 256 * 256)
    if (N - 1) * K * 2 + 2 * K <= _U32 and N * K < 2 ** 31:
        return rc, N
    unit = 256
    while (unit * K) % blocksize:
        unit *= 2
    nc = min((_U32 - 2 * K) // (2 * K) + 1, (2 ** 31 - 1) // K) // unit * unit
    return rc, max(unit, nc)


def _gemm_4bit_hgemm_chunked(A2: Tensor, Bc: Tensor, state: QuantState, out: Tensor,
                             absmax: Optional[Tensor]) -> Tensor:
    """dequantise + k_hgemm for operands beyond one launch's 32-bit offsets (previously the library
    GEMM): the weight is dequantised one row chunk at a time into the weight workspace, and each weight chunk is
    multiplied with each activation row chunk straight into its [rows, columns] block of `out` (ldc = N).  Every output
    element is one k_hgemm dot product over all of K, as in the one-launch form (the plan per chunk shape may split K
    differently, within the GEMM tolerance)."""
    rows, K = A2.shape
    N = state.shape[0]
    rc, nc = _hgemm_chunks(rows, N, K, state.blocksize)
    am = absmax if absmax is not None else _absmax_fp32(state)
    bs = state.blocksize
    qt = "fp4" if state.quant_type == "fp4" else "nf4"
    deq = getattr(lib, f"cdequantize_blockwise_{_QB[A2.dtype]}_{qt}")
    gemm = lib.chgemm_tn_ws_bf16 if A2.dtype == torch.bfloat16 else lib.chgemm_tn_ws_fp16
    flat = Bc.reshape(-1)
    outv = out.view(rows, N)
    for n0 in range(0, N, nc):
        n1 = min(N, n0 + nc)
        W = _dequant_workspace(A2.device, A2.dtype, (n1 - n0) * K).view(n1 - n0, K)
        prev_device = pre_call(A2.device)
        deq(get_ptr(None), get_ptr(flat[n0 * K // 2:]), get_ptr(am[n0 * K // bs:]), get_ptr(W), ct.c_int(bs),
            ct.c_int((n1 - n0) * K))
        _DEQ_META.pop((A2.device, A2.dtype, _stream_key(A2.device)), None)   # the workspace holds a chunk now
        for r0 in range(0, rows, rc):
            r1 = min(rows, r0 + rc)
            ws_bytes = int(lib.chgemm_tn_workspace_bytes(ct.c_int32(r1 - r0), ct.c_int32(n1 - n0), ct.c_int32(K)))
            ws = _gemm_workspace(A2.device, ws_bytes)
            rc_ = gemm(ct.c_int32(r1 - r0), ct.c_int32(n1 - n0), ct.c_int32(K), get_ptr(A2[r0:]), ct.c_int32(K),
                       get_ptr(W), ct.c_int32(K), get_ptr(outv[r0:, n0:]), ct.c_int32(N), get_ptr(ws),
                       ct.c_longlong(ws_bytes))
            if rc_:
                post_call(prev_device)
                raise RuntimeError(f"bitsandbytes HIP GEMM (chgemm_tn, chunk rows {r0}:{r1} x features {n0}:{n1}) "
                                   f"returned {rc_}: " + (lib.cget_last_error_message().decode() if rc_ == 2
                                                          else "shape not supported"))
        post_call(prev_device)
    return out


def gemm_4bit_static_route(rows: int, N: int, K: int) -> str:
    """The deterministic route of a (rows, N, K) product (round 4, tools/route_sweep4.py, profiles/lab/r04_route_sweep.txt):
      * up to GEMM_4BIT_FEW_TOKENS rows: "fused" (the few-token kernels and the multi-row GEMV, picked inside);
      * the one-kernel fused NF4 GEMM ("fused") where the weight is deep and wide and the rows few -- K >= 8192 and
        N >= 4096 up to 384 rows (4096 x 11008 at 96..256 rows 45-55 us vs 50-59 dequantise + k_hgemm; 8192 x 8192
        52-65 vs 62-86), K >= 16384 at 513..1024 rows (1024 x 28672 at 1024 rows 84 vs 100): there the bf16 weight's
        write + read costs more than the fused kernel's in-LDS dequantisation.  Round 5 (the 128 x 128 k_hgemm tile,
        profiles/lab/r05_route_sweep.txt): at 512 rows the pair is ahead or level (4096 x 11008 73-80 vs 81; 8192 x
        8192 97 vs 97; 1024 x 28672 64 vs 69), so the band ends at 384 / starts above 512;
      * everywhere else the dequantise + the hand-written k_hgemm ("hgemm"; 256 x 256 / 256 x 128 / 128 x 256 tiles and
        split-K by its launch plan); operands beyond one launch's 32-bit offsets (prompts above ~195k tokens at K =
        11008, weights above 2^31 elements) run it in row / weight chunks (_gemm_4bit_hgemm_chunked).  "library" only
        for K % 64 != 0, which gemm_4bit does not take (gemm_4bit_supported): no vendor GEMM on the static route.
    Accepted trade: 65..256 rows of wide weights (11008 x 4096 at 96 / 128 / 256 rows) run 5-8 % slower on
    k_hgemm than on the library GEMM (52.5 / 54.0 / 60.4 vs 48.9 / 51.8 / 58.7 us, profiles/lab/r04_route_sweep.txt);
    BNB_ROUTE_TUNING=1 measures and picks the faster route per shape."""
    if rows <= GEMM_4BIT_FEW_TOKENS:
        return "fused"
    if rows < GEMM_4BIT_DEQUANT_MIN_ROWS:
        if (K >= 8192 and N >= 4096 and rows <= 384) or (K >= 16384 and 512 < rows <= 1024):
            return "fused"
    return "hgemm" if K % 64 == 0 else "library"


def _tuned_route(A2: Tensor, Bc: Tensor, state: QuantState, out: Tensor, absmax: Optional[Tensor],
                 default: str) -> str:
    """The measured route of a prefill shape (see above); `default` is the static rule's route, kept unless another
    is faster by more than GEMM_4BIT_ROUTE_MARGIN.  Timed on A2's device and its current stream."""
    _load_route_plan()
    key = _route_key(A2, state, absmax)
    route = _ROUTES.get(key)
    if route is not None:
        return route
    with torch.cuda.device(A2.device):
        stream = torch.cuda.current_stream(A2.device)
        if torch.cuda.is_current_stream_capturing():
            return default
        ws_key = (A2.device, A2.dtype, _stream_key(A2.device))
        ws_before = _DEQ_WS.get(ws_key)
        rows, N, K = A2.shape[0], state.shape[0], state.shape[1]
        # "hgemm" is always a candidate (gemm_4bit runs it in row / weight chunks beyond one launch's offsets); the
        # library candidates dequantise the whole weight with a 32-bit element count, so not from 2^31 elements on
        big = N * K >= 2 ** 31
        names = [n for n in GEMM_4BIT_ROUTES if not (big and n in ("library", "library_tn"))]
        for name in names:      # untimed: code-object loads, the rocBLAS solution search, workspaces, clock ramp
            gemm_4bit(A2, Bc, state, out=out, absmax=absmax, _route=name)
        times = {name: float("inf") for name in names}
        for _ in range(3):      # interleaved rounds, best per route (no route is timed only on a colder clock)
            for name in names:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record(stream)
                gemm_4bit(A2, Bc, state, out=out, absmax=absmax, _route=name)
                e.record(stream)
                e.synchronize()
                times[name] = min(times[name], s.elapsed_time(e))
        fastest = min(times, key=times.get)
        route = fastest if times[fastest] < (1.0 - GEMM_4BIT_ROUTE_MARGIN) * times.get(default, float("inf")) else default
        if route == "fused" and _DEQ_WS.get(ws_key) is not ws_before:
            # the library candidates grew the weight workspace for this measurement only: give it back
            if ws_before is None:
                _DEQ_WS.pop(ws_key, None)
            else:
                _DEQ_WS[ws_key] = ws_before
            _DEQ_META.pop(ws_key, None)
    _ROUTES[key] = route
    _save_route_plan()
    return route


def _dequant_workspace(device, dtype, numel: int) -> Tensor:
    """Grow-only weight buffer per (device, dtype, stream) for the dequantise + library-GEMM path (the
    size of the largest weight seen; per stream, so concurrent streams never share one)."""
    key = (device, dtype, _stream_key(device))
    ws = _DEQ_WS.get(key)
    if ws is None or ws.numel() < numel:
        ws = torch.empty(numel, dtype=dtype, device=device)
        _DEQ_WS[key] = ws
        _DEQ_META.pop(key, None)
    return ws[:numel]


def _fewtok_takes(n: int, rows: int, k: int, blocksize: int) -> bool:
    """Whether the C side runs the whole-K few-token kernel (gemm4bit_fewtok.hip) for this shape; 2..4 rows then go
    there instead of the multi-row GEMV (measured faster wherever its rule takes the shape, profiles/lab/r03_fewtok32.txt).
    Asked on every call (one cheap ctypes call, 2..4-row products only): the C answer applies the same conditions as the
    launch, including every A/B knob (fewtok mode, the older few-token kernels, the split-K geometry), so no cached
    answer can go stale when a knob changes."""
    return bool(lib.cgemm_4bit_fewtok_takes(ct.c_int32(n), ct.c_int32(rows), ct.c_int32(k), ct.c_int32(blocksize)))


_FEWTOK_MODE = [0]


def set_fewtok_mode(mode: int) -> None:
    """Test / A-B knob of the whole-K few-token kernel: 0 = auto, 1 = off, 2 = wherever it fits."""
    lib.cgemm_4bit_set_fewtok_mode(ct.c_int(mode))
    _FEWTOK_MODE[0] = mode


_EVENT_POOL: list = []


def reserve_stage_events(n: int) -> None:
    """Pre-create n timing events for the `events=` instrumentation of gemm_4bit (bench): creating them inside a timed
    step costs host time that can leave the GPU waiting in exactly the steps that are sampled."""
    for _ in range(n):
        e = torch.cuda.Event(enable_timing=True)
        e.record()                         # the HIP event itself is created at its first record
        _EVENT_POOL.append(e)
    torch.cuda.synchronize()


def _stage_events(n: int) -> list:
    return [_EVENT_POOL.pop() if _EVENT_POOL else torch.cuda.Event(enable_timing=True) for _ in range(n)]


def _gemm_4bit_tokens(A2: Tensor, Bc: Tensor, state: QuantState, out: Tensor, absmax: Optional[Tensor],
                      events: Optional[list]) -> bool:
    """2..GEMM_4BIT_GEMV_TOKENS rows through cgemm_4bit_inference_tokens_* (one launch; compressed statistics
    decoded in the kernel).  False when the entry point declines the shape (nothing launched)."""
    N, K = state.shape[0], state.shape[1]
    rows = A2.shape[0]
    nested = absmax is None and _nested_stats_in_kernel_ok(state)
    if nested:
        s2 = state.state2
        stats = [None, state.absmax, s2.code, s2.absmax, _offset_on(state, A2.device)]
        bs2 = s2.blocksize
    else:
        stats = [absmax if absmax is not None else _absmax_fp32(state), None, None, None, None]
        bs2 = 0
    prev_device = pre_call(A2.device)
    is_on_gpu([A2, Bc, out, state.code] + [t for t in stats if t is not None])
    ev = _stage_events(2) if events is not None else None
    if ev:
        ev[0].record()
    fn = lib.cgemm_4bit_inference_tokens_bf16 if A2.dtype == torch.bfloat16 else lib.cgemm_4bit_inference_tokens_fp16
    rc = fn(ct.c_int32(N), ct.c_int32(rows), ct.c_int32(K), get_ptr(A2), ct.c_int32(K), get_ptr(Bc),
            ct.c_int32((K + 1) // 2), *[get_ptr(t) for t in stats], get_ptr(state.code), get_ptr(out), ct.c_int32(N),
            ct.c_int32(state.blocksize), ct.c_int32(bs2))
    post_call(prev_device)
    if rc == 2:
        raise RuntimeError(f"bitsandbytes HIP kernel error: {lib.cget_last_error_message().decode()}")
    if rc == 0 and ev:
        ev[1].record()
        events.append(("gemm", ev[0], ev[1]))
    return rc == 0


# Prefetched weights (gemm_4bit(..., prefetch=...)): per (device, dtype, stream) two weight slots and the slot + identity
# of the weight the last prefetching GEMM dequantised into one of them.
_PF_WS: dict = {}
_PF_READY: dict = {}
_PF_CUR: dict = {}          # the slot + identity the last consuming call read (reuse_weight chunks read it again)


def _weight_meta(B: Tensor, state: QuantState, absmax: Optional[Tensor]) -> tuple:
    """What identifies a dequantised weight: the packed bytes and the statistics (pointers and versions), shape,
    blocksize and code -- the same tuple whether the weight is dequantised by its own call or prefetched."""
    stats = absmax if absmax is not None else state.absmax
    return (B.data_ptr(), B._version, stats.data_ptr(), stats._version, state.shape[0], state.shape[1], state.blocksize,
            state.quant_type)


def _pf_slots(key, device, dtype, numel: int) -> list:
    slots = _PF_WS.get(key)
    if slots is None or slots[0].numel() < numel:
        slots = [torch.empty(numel, dtype=dtype, device=device) for _ in range(2)]
        _PF_WS[key] = slots
        _PF_READY.pop(key, None)
        _PF_CUR.pop(key, None)
    return slots


def prefetched_weight(device, dtype=torch.bfloat16) -> Optional[tuple]:
    """(slot, identity) of the weight waiting in a prefetch slot on this device / dtype / current stream, or None."""
    return _PF_READY.get((torch.device(device), dtype, _stream_key(torch.device(device))))


def _launch_prefetch_gemm(A2: Tensor, W: Tensor, out: Tensor, ws: Optional[Tensor], ws_bytes: int, pf: tuple,
                          target: Tensor) -> int:
    """chgemm_tn_pf_*: the GEMM of this call with the next weight's dequantise (pf = (B_next, state_next[, absmax]))
    into `target` inside it.  Returns the C code (0 launched, 1 not supported -- nothing launched, 2 error)."""
    Bn, sn = pf[0], pf[1]
    an = pf[2] if len(pf) > 2 else None
    rows, K = A2.shape
    N = W.shape[0]
    nested = an is None and sn.nested and _nested_stats_in_kernel_ok(sn)
    if nested:
        s2 = sn.state2
        stats = [None, sn.absmax, s2.code, s2.absmax, _offset_on(sn, A2.device)]
        bs2 = s2.blocksize
    else:
        stats = [an if an is not None else _absmax_fp32(sn), None, None, None, None]
        bs2 = 0
    Bc = Bn                      # (contiguous: gemm_4bit drops the hint otherwise)
    is_on_gpu([Bc, target] + [t for t in stats if t is not None])
    fn = lib.chgemm_tn_pf_bf16 if A2.dtype == torch.bfloat16 else lib.chgemm_tn_pf_fp16
    return fn(ct.c_int32(rows), ct.c_int32(N), ct.c_int32(K), get_ptr(A2), ct.c_int32(K), get_ptr(W), ct.c_int32(K),
              get_ptr(out), ct.c_int32(N), get_ptr(ws), ct.c_longlong(ws_bytes), get_ptr(Bc),
              *[get_ptr(t) for t in stats], ct.c_int32(1 if sn.quant_type == "fp4" else 0), ct.c_int32(sn.blocksize),
              ct.c_int32(bs2), ct.c_longlong(sn.shape[0] * sn.shape[1]), get_ptr(target))


def gemm_4bit(A: Tensor, B: Tensor, state: QuantState, out: Optional[Tensor] = None,
              absmax: Optional[Tensor] = None, events: Optional[list] = None, reuse_weight: bool = False,
              _route: Optional[str] = None, prefetch: Optional[tuple] = None) -> Tensor:
    """4-bit weight GEMM for any number of activation rows (the M>1 slot of cgemm_4bit_inference,
    ref:pythonInterface.cpp:377).  out[..., n] = A[..., :] @ W^T with W the dequantised [N, K] weight;
    replaces dequantize_4bit + F.linear (autograd/_functions.py:507).  The route per shape is
    gemm_4bit_static_route: from 65 rows (outside the fused-kernel band) the HIP dequantise kernel into a weight
    workspace + the hand-written k_hgemm (hgemm.hip; chunked beyond one launch's 32-bit offsets), otherwise the
    few-token kernels or the fused kernel (dequantise in LDS + MFMA, split-K when the tile grid is small).
    B is the packed uint8 weight (any view of the N*K/2 bytes).  events (bench instrumentation): a list
    that receives (name, start, end) torch.cuda.Event pairs around the launched stages.  reuse_weight:
    the caller runs several row chunks of one product against the same, unmodified weight (the chunked
    sharded forward); on the library path the workspace still holding this weight's dequantisation
    from the previous call is used as is.  Prefill shapes on the library side of the static rule take the
    measured route (GEMM_4BIT_ROUTE_TUNING); _route (one of GEMM_4BIT_ROUTES) forces one (internal).
    prefetch = (B_next, state_next[, absmax_next]): the weight of the NEXT gemm_4bit call on this stream (the layer's
    next projection, the next layer's first): on the dequantise + k_hgemm route its dequantise runs inside this call's
    GEMM (chgemm_tn_pf_*, hgemm.hip HgSide) into a second weight slot, and the next call whose weight it is finds it
    there and launches the GEMM alone -- the dequantise software-pipelined one weight ahead, the same bits as the
    unpipelined pair.  On other routes the hint is ignored (the next call dequantises its own weight)."""
    if not gemm_4bit_supported(A, state):
        raise ValueError("gemm_4bit: needs bf16/fp16 activations and in_features % 64 == 0")
    N, K = state.shape[0], state.shape[1]
    A2 = A.reshape(-1, K)
    if not A2.is_contiguous() or A2.data_ptr() % 16:
        A2 = A2.contiguous()
    rows = A2.shape[0]
    if out is None:
        out = torch.empty((rows, N), dtype=A.dtype, device=A.device)
    Bc = B if B.is_contiguous() else B.contiguous()
    if prefetch is not None and not prefetch[0].is_contiguous():
        # the prefetched weight is matched to its consuming call by the packed bytes' pointer and version: a temporary
        # contiguous copy would be freed at once and its address reused, so the hint needs B_next in place
        prefetch = None
    route = gemm_4bit_static_route(rows, N, K)
    if _route is not None:
        if _route not in GEMM_4BIT_ROUTES:
            raise ValueError(f"gemm_4bit: unknown route {_route!r}")
        route = _route
    elif GEMM_4BIT_ROUTE_TUNING and rows > GEMM_4BIT_FEW_TOKENS:
        route = _tuned_route(A2, Bc, state, out.view(rows, N), absmax, route)
    elif rows > GEMM_4BIT_FEW_TOKENS and (_ROUTES or _plan_path()):
        measured = gemm_4bit_measured_route(A2, state, absmax)   # a table handed over by import_routes / the plan file
        if measured is not None:
            route = measured
    if route == "hgemm" and not _hgemm_fits(rows, N, K):
        # beyond one launch's 32-bit offsets: the same pair in row / weight chunks (also where a measured / imported
        # route, which covers a quarter-octave of row counts, names "hgemm" near the limit).  reuse_weight and prefetch
        # do not apply there (each call dequantises its weight chunk by chunk); events get one "gemm" pair around it all
        ev = _stage_events(2) if events is not None else None
        if ev:
            ev[0].record()
        _gemm_4bit_hgemm_chunked(A2, Bc, state, out, absmax)
        if ev:
            ev[1].record()
            events.append(("gemm", ev[0], ev[1]))
        return out.view(*A.shape[:-1], N)
    library = route in ("library", "library_tn", "hgemm")
    if (not library and 2 <= rows <= GEMM_4BIT_GEMV_TOKENS and not _fewtok_takes(N, rows, K, state.blocksize)
            and _gemm_4bit_tokens(A2, Bc, state, out, absmax, events)):
        return out.view(*A.shape[:-1], N)
    if (absmax is None and not library and rows <= GEMM_4BIT_FEW_TOKENS and _nested_stats_in_kernel_ok(state)):
        # few tokens, compressed statistics: one launch of the weight-streaming kernel that decodes the
        # nested absmax in-kernel (no separate decode launch)
        ws_bytes = int(lib.cgemm_4bit_workspace_bytes(ct.c_int32(N), ct.c_int32(rows), ct.c_int32(K)))
        ws = _gemm_workspace(A.device, ws_bytes)
        s2 = state.state2
        offset = _offset_on(state, A.device)
        prev_device = pre_call(A.device)
        is_on_gpu([A2, Bc, out, state.absmax, s2.code, s2.absmax, offset, state.code])
        ev = _stage_events(2) if events is not None else None
        if ev:
            ev[0].record()
        fn = (lib.cgemm_4bit_inference_nested_ws_bf16 if A.dtype == torch.bfloat16
              else lib.cgemm_4bit_inference_nested_ws_fp16)
        rc = fn(ct.c_int32(N), ct.c_int32(rows), ct.c_int32(K), get_ptr(A2), get_ptr(Bc), get_ptr(state.absmax),
                get_ptr(s2.code), get_ptr(s2.absmax), get_ptr(offset), get_ptr(state.code), get_ptr(out),
                ct.c_int32(K), ct.c_int32((K + 1) // 2), ct.c_int32(N), ct.c_int32(state.blocksize),
                ct.c_int32(s2.blocksize), get_ptr(ws), ct.c_longlong(ws_bytes))
        if rc == 0:
            post_call(prev_device)
            if ev:
                ev[1].record()
                events.append(("gemm", ev[0], ev[1]))
            return out.view(*A.shape[:-1], N)
        post_call(prev_device)
    if absmax is None and not (library and state.nested):
        absmax = _absmax_fp32(state)
    prev_device = pre_call(A.device)
    is_on_gpu([A2, Bc, out, state.code] + ([absmax] if absmax is not None else []))
    ev = _stage_events(3) if events is not None else None
    if ev:
        ev[0].record()
    if library:
        key = (A.device, A.dtype, _stream_key(A.device))
        meta = _weight_meta(Bc, state, absmax)
        ready = _PF_READY.get(key)
        cur_slot = None
        if ready is not None and ready[1] == meta:
            # dequantised by the previous call's GEMM (prefetch): consumed here (row chunks of this same product that
            # follow with reuse_weight read it again, until a prefetch overwrites the slot)
            cur_slot = ready[0]
            del _PF_READY[key]
            _PF_CUR[key] = ready
        elif reuse_weight and _PF_CUR.get(key, (None, None))[1] == meta:
            cur_slot = _PF_CUR[key][0]
        if cur_slot is not None:
            W = _PF_WS[key][cur_slot][:N * K].view(N, K)
        else:
            W = _dequant_workspace(A.device, A.dtype, N * K).view(N, K)
        if cur_slot is None and not (reuse_weight and _DEQ_META.get(key) == meta):
            if absmax is None and not _dequant_4bit_nested(Bc, state, W):   # nested stats decoded in-kernel
                absmax = _absmax_fp32(state)
            if absmax is not None:
                qt = "fp4" if state.quant_type == "fp4" else "nf4"
                getattr(lib, f"cdequantize_blockwise_{_QB[A.dtype]}_{qt}")(
                    get_ptr(None), get_ptr(Bc), get_ptr(absmax), get_ptr(W), ct.c_int(state.blocksize),
                    ct.c_int(N * K))
            _DEQ_META[key] = meta
            if ev:
                ev[1].record()
                events.append(("dequantize", ev[0], ev[1]))
        elif ev:
            ev[1].record()
        if route == "hgemm":
            # the hand-written GEMM (hgemm.hip); split-K over a workspace on small tile grids (chgemm_tn_ws_*)
            ws_bytes = int(lib.chgemm_tn_workspace_bytes(ct.c_int32(rows), ct.c_int32(N), ct.c_int32(K)))
            ws = _gemm_workspace(A.device, ws_bytes)
            rc = 1
            if prefetch is not None:
                sn = prefetch[1]
                nn = sn.shape[0] * sn.shape[1]
                # (if the slots are re-made larger here, W still holds the old slot this call reads; both new ones
                # are free)
                slots = _pf_slots(key, A.device, A.dtype, max(nn, N * K))
                target = 1 - cur_slot if cur_slot is not None else 0
                rc = _launch_prefetch_gemm(A2, W, out, ws, ws_bytes, prefetch, slots[target][:nn])
                if rc == 0:
                    if _PF_CUR.get(key, (None,))[0] == target:
                        _PF_CUR.pop(key, None)
                    _PF_READY[key] = (target, _weight_meta(prefetch[0], sn, prefetch[2] if len(prefetch) > 2 else None))
            if rc == 1:
                fn = lib.chgemm_tn_ws_bf16 if A.dtype == torch.bfloat16 else lib.chgemm_tn_ws_fp16
                rc = fn(ct.c_int32(rows), ct.c_int32(N), ct.c_int32(K), get_ptr(A2), ct.c_int32(K), get_ptr(W),
                        ct.c_int32(K), get_ptr(out), ct.c_int32(N), get_ptr(ws), ct.c_longlong(ws_bytes))
            post_call(prev_device)
            if rc:
                raise RuntimeError(f"bitsandbytes HIP GEMM (chgemm_tn) returned {rc}: "
                                   f"{lib.cget_last_error_message().decode() if rc == 2 else 'shape not supported'}")
        elif route == "library_tn":
            # the library GEMM with the per-shape solution search (gemm_lib.hip, rocBLAS)
            fn = lib.cgemm_tn_bf16 if A.dtype == torch.bfloat16 else lib.cgemm_tn_fp16
            rc = fn(ct.c_int32(rows), ct.c_int32(N), ct.c_int32(K), get_ptr(A2), ct.c_int32(K), get_ptr(W),
                    ct.c_int32(K), get_ptr(out), ct.c_int32(N))
            post_call(prev_device)
            if rc:
                raise RuntimeError(f"bitsandbytes HIP library GEMM error: {lib.cget_last_error_message().decode()}")
        else:
            post_call(prev_device)
            torch.matmul(A2, W.t(), out=out.view(rows, N))
        if ev:
            ev[2].record()
            events.append(("gemm", ev[1], ev[2]))
        return out.view(*A.shape[:-1], N)
    ws_bytes = int(lib.cgemm_4bit_workspace_bytes(ct.c_int32(N), ct.c_int32(rows), ct.c_int32(K)))
    ws = _gemm_workspace(A.device, ws_bytes)
    fn = lib.cgemm_4bit_inference_code_ws_bf16 if A.dtype == torch.bfloat16 else lib.cgemm_4bit_inference_code_ws_fp16
    fn(ct.c_int32(N), ct.c_int32(rows), ct.c_int32(K), get_ptr(A2), get_ptr(Bc), get_ptr(absmax),
       get_ptr(state.code), get_ptr(out), ct.c_int32(K), ct.c_int32((K + 1) // 2), ct.c_int32(N),
       ct.c_int32(state.blocksize), get_ptr(ws), ct.c_longlong(ws_bytes))
    post_call(prev_device)
    if ev:
        ev[2].record()
        events.append(("gemm", ev[0], ev[2]))
    return out.view(*A.shape[:-1], N)


# ----------------------------------------------------------------------------- LLM.int8
def get_transform_buffer(shape, dtype, device, to_order, from_order="row", transpose=False):
    """ref:functional.py:482-518"""
    init_func = torch.zeros
    dims = len(shape)
    if dims == 2:
        rows = shape[0]
    elif dims == 3:
        rows = shape[0] * shape[1]
    cols = shape[-1]
    state = (shape, to_order)
    if transpose:
        rows, cols = cols, rows
        state = (shape[::-1], to_order)
    if to_order == "row" or to_order == "col":
        return init_func(shape, dtype=dtype, device=device), state
    elif to_order == "col32":
        cols = 32 * ((cols + 31) // 32)
        return init_func((rows, cols), dtype=dtype, device=device), state
    elif to_order == "col_turing":
        cols = 32 * ((cols + 31) // 32)
        rows = 8 * ((rows + 7) // 8)
        return init_func((rows, cols), dtype=dtype, device=device), state
    elif to_order == "col_ampere":
        cols = 32 * ((cols + 31) // 32)
        rows = 32 * ((rows + 31) // 32)
        return init_func((rows, cols), dtype=dtype, device=device), state
    raise NotImplementedError(f"To_order not supported: {to_order}")


def transform(A, to_order, from_order="row", out=None, transpose=False, state=None, ld=None):
    """Row-major int8 <-> col32 / col_turing / col_ampere tiles (ref:functional.py:2607-2653)."""
    prev_device = pre_call(A.device)
    if state is None:
        state = (A.shape, from_order)
    else:
        from_order = state[1]
    if out is None:
        if to_order == "row":
            out, new_state = torch.empty(state[0], dtype=A.dtype, device=A.device), (state[0], "row")
        else:
            out, new_state = get_transform_buffer(state[0], A.dtype, A.device, to_order, state[1], transpose)
    else:
        new_state = (state[0], to_order)
    shape = state[0]
    if len(shape) == 2:
        dim1, dim2 = ct.c_int32(shape[0]), ct.c_int32(shape[1])
    else:
        dim1, dim2 = ct.c_int32(shape[0] * shape[1]), ct.c_int32(shape[2])
    is_on_gpu([A, out])
    if to_order == "col32":
        (lib.ctransform_row2col32T if transpose else lib.ctransform_row2col32)(get_ptr(A), get_ptr(out), dim1, dim2)
    elif to_order == "col_turing":
        (lib.ctransform_row2turingT if transpose else lib.ctransform_row2turing)(get_ptr(A), get_ptr(out), dim1, dim2)
    elif to_order == "col_ampere":
        (lib.ctransform_row2ampereT if transpose else lib.ctransform_row2ampere)(get_ptr(A), get_ptr(out), dim1, dim2)
    elif to_order == "row":
        if from_order == "col_turing":
            lib.ctransform_turing2row(get_ptr(A), get_ptr(out), dim1, dim2)
        elif from_order == "col_ampere":
            lib.ctransform_ampere2row(get_ptr(A), get_ptr(out), dim1, dim2)
        elif from_order == "col32":
            lib.ctransform_col322row(get_ptr(A), get_ptr(out), dim1, dim2)
        else:
            raise NotImplementedError(f"Transform function not implemented: From {from_order} to {to_order}")
    else:
        raise NotImplementedError(f"Transform function not implemented: From {from_order} to {to_order}")
    post_call(prev_device)
    return out, new_state


def igemmlt(A, B, SA, SB, out=None, Sout=None, dtype=torch.int32):
    """C = A @ B^T on int8 tiles, int32 (or int8) col32 output (ref:functional.py:2260-2352)."""
    shapeA, shapeB = SA[0], SB[0]
    dimsA, dimsB = len(shapeA), len(shapeB)
    assert dimsB == 2, "Only two dimensional matrices are supported for argument B"
    if dimsA == 2:
        m = shapeA[0]
    elif dimsA == 3:
        m = shapeA[0] * shapeA[1]
    rows = n = shapeB[0]
    assert prod(list(shapeA)) > 0, f"Input tensor dimensions need to be > 0: {shapeA}"
    if shapeA[0] == 0 and dimsA == 2:
        return torch.empty((0, shapeB[0]), device=A.device, dtype=torch.float16)
    elif shapeA[1] == 0 and dimsA == 3:
        return torch.empty(tuple(shapeA[:2] + [shapeB[0]]), device=A.device, dtype=torch.float16)
    if dimsA == 2 and out is None:
        out, Sout = get_transform_buffer((shapeA[0], shapeB[0]), dtype, A.device, "col32", "row")
    elif dimsA == 3 and out is None:
        out, Sout = get_transform_buffer((shapeA[0], shapeA[1], shapeB[0]), dtype, A.device, "col32", "row")
    assert dimsB != 3, "len(B.shape)==3 not supported"
    assert A.device.type == "cuda" and B.device.type == "cuda"
    assert A.dtype == torch.int8 and B.dtype == torch.int8
    assert out.dtype == dtype
    assert SA[1] == "col32"
    assert SB[1] in ["col_turing", "col_ampere"]
    assert Sout[1] == "col32"
    assert shapeA[-1] == shapeB[-1], (
        f"Matmullt only supports A @ B^T. Inner matrix dimensions do not match: A @ B = {shapeA} @ {shapeB}")
    formatB = SB[1]
    prev_device = pre_call(A.device)
    k = shapeA[-1]
    lda = ct.c_int32(m * 32)
    if formatB == "col_turing":
        ldb = ct.c_int32(((rows + 7) // 8) * 8 * 32)
    else:
        ldb = ct.c_int32(((rows + 31) // 32) * 32 * 32)
    ldc = ct.c_int32(m * 32)
    is_on_gpu([A, B, out])
    fmt = "turing" if formatB == "col_turing" else "ampere"
    fn = getattr(lib, f"cigemmlt_{fmt}_32" if dtype == torch.int32 else f"cigemmlt_{fmt}_8")
    has_error = fn(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k), get_ptr(A), get_ptr(B), get_ptr(out), get_ptr(None),
                   lda, ldb, ldc)
    if has_error == 1:
        has_error = 100
    if has_error == 100:
        raise NotImplementedError("igemmlt not available (probably built with NO_CUBLASLT)")
    if has_error:
        raise Exception("igemmlt ran into an error!")
    post_call(prev_device)
    return out, Sout


def mm_dequant(A, quant_state, row_stats, col_stats, out=None, new_row_stats=None, new_col_stats=None, bias=None):
    """int32 col32 -> fp16 row-major with row/col stats and bias (ref:functional.py:2355-2397)."""
    assert A.dtype == torch.int32
    if bias is not None:
        assert bias.dtype == torch.float16
    out_shape = quant_state[0]
    if len(out_shape) == 3:
        out_shape = (out_shape[0] * out_shape[1], out_shape[2])
    if out is None:
        out = torch.empty(out_shape, dtype=torch.float16, device=A.device)
    if new_row_stats is None:
        new_row_stats = torch.empty(out_shape[0], dtype=torch.float32, device=A.device)
    if new_col_stats is None:
        new_col_stats = torch.empty(out_shape[1], dtype=torch.float32, device=A.device)
    assert new_row_stats.shape[0] == row_stats.shape[0], f"{new_row_stats.shape} vs {row_stats.shape}"
    assert new_col_stats.shape[0] == col_stats.shape[0], f"{new_col_stats.shape} vs {col_stats.shape}"
    prev_device = pre_call(A.device)
    is_on_gpu([A, row_stats, col_stats, out, new_row_stats, new_col_stats, bias])
    lib.cdequant_mm_int32_fp16(get_ptr(A), get_ptr(row_stats), get_ptr(col_stats), get_ptr(out),
                               get_ptr(new_row_stats), get_ptr(new_col_stats), get_ptr(bias),
                               ct.c_int32(out_shape[0]), ct.c_int32(out_shape[1]))
    post_call(prev_device)
    return out


def igemmlt_dequant(CA: Tensor, CB: Tensor, row_stats: Tensor, col_stats: Tensor, bias: Optional[Tensor] = None,
                    out: Optional[Tensor] = None) -> Tensor:
    """Fused LLM.int8 matmul on row-major int8 operands: mm_dequant(igemmlt(CA, CB)) in one launch
    (additive entry point cigemmlt_row_dequant_fp16).  CA [m, k] int8, CB [n, k] int8 -> fp16 [m, n]."""
    assert CA.dtype == torch.int8 and CB.dtype == torch.int8
    m, k = CA.reshape(-1, CA.shape[-1]).shape
    n = CB.shape[0]
    assert CB.shape[1] == k
    if bias is not None:
        assert bias.dtype == torch.float16
    CA2 = CA.reshape(m, k).contiguous()
    CBc = CB.contiguous()
    if out is None:
        out = torch.empty((m, n), dtype=torch.float16, device=CA.device)
    # small tile grids (the column shards of the multi-GPU step) run split-K through the grow-only workspace
    ws_bytes = int(lib.cigemmlt_workspace_bytes(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k)))
    ws = _gemm_workspace(CA.device, ws_bytes)
    prev_device = pre_call(CA.device)
    is_on_gpu([CA2, CBc, row_stats, col_stats, out, bias])
    err = lib.cigemmlt_row_dequant_ws_fp16(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k), get_ptr(CA2), get_ptr(CBc),
                                           get_ptr(out), get_ptr(row_stats), get_ptr(col_stats), get_ptr(bias),
                                           ct.c_int32(k), ct.c_int32(k), ct.c_int32(n), get_ptr(ws),
                                           ct.c_longlong(ws_bytes))
    if err:
        raise Exception("igemmlt ran into an error!")
    post_call(prev_device)
    return out


def igemm_rowmajor(A: Tensor, B: Tensor, out: Optional[Tensor] = None) -> Tensor:
    """Exact int8 x int8 -> int32, C = A @ B^T on row-major operands (additive cigemm_row_i32)."""
    m, k = A.shape
    n = B.shape[0]
    if out is None:
        out = torch.empty((m, n), dtype=torch.int32, device=A.device)
    ws_bytes = int(lib.cigemmlt_workspace_bytes(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k)))
    ws = _gemm_workspace(A.device, ws_bytes)
    Ac, Bc = A.contiguous(), B.contiguous()
    prev_device = pre_call(A.device)
    is_on_gpu([A, B, out])
    err = lib.cigemm_row_i32_ws(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k), get_ptr(Ac), get_ptr(Bc), get_ptr(out),
                                ct.c_int32(k), ct.c_int32(k), ct.c_int32(n), get_ptr(ws), ct.c_longlong(ws_bytes))
    if err:
        raise Exception("igemm ran into an error!")
    post_call(prev_device)
    return out


def get_colrow_absmax(A, row_stats=None, col_stats=None, nnz_block_ptr=None, threshold=0.0):
    """Row and column absmax of an fp16 matrix (ref:functional.py:2400-2435)."""
    assert A.dtype == torch.float16
    device = A.device
    cols = A.shape[-1]
    rows = A.shape[0] * A.shape[1] if len(A.shape) == 3 else A.shape[0]
    col_tiles = (cols + 255) // 256
    tiled_rows = ((rows + 15) // 16) * 16
    if row_stats is None:
        row_stats = torch.empty((rows,), dtype=torch.float32, device=device).fill_(-50000.0)
    if col_stats is None:
        col_stats = torch.empty((cols,), dtype=torch.float32, device=device).fill_(-50000.0)
    if nnz_block_ptr is None and threshold > 0.0:
        nnz_block_ptr = torch.zeros(((tiled_rows * col_tiles) + 1,), dtype=torch.int32, device=device)
    prev_device = pre_call(A.device)
    is_on_gpu([A, row_stats, col_stats, nnz_block_ptr])
    lib.cget_col_row_stats(get_ptr(A), get_ptr(row_stats), get_ptr(col_stats), get_ptr(nnz_block_ptr),
                           ct.c_float(threshold), ct.c_int32(rows), ct.c_int32(cols))
    post_call(prev_device)
    if threshold > 0.0:
        nnz_block_ptr.cumsum_(0)
    return row_stats, col_stats, nnz_block_ptr


class COOSparseTensor:
    def __init__(self, rows, cols, nnz, rowidx, colidx, values):
        assert rowidx.dtype == torch.int32 and colidx.dtype == torch.int32 and values.dtype == torch.float16
        assert values.numel() == nnz and rowidx.numel() == nnz and colidx.numel() == nnz
        self.rows, self.cols, self.nnz = rows, cols, nnz
        self.rowidx, self.colidx, self.values = rowidx, colidx, values


def coo_zeros(rows, cols, nnz, device, dtype=torch.half):
    rowidx = torch.zeros((nnz,), dtype=torch.int32, device=device)
    colidx = torch.zeros((nnz,), dtype=torch.int32, device=device)
    values = torch.zeros((nnz,), dtype=dtype, device=device)
    return COOSparseTensor(rows, cols, nnz, rowidx, colidx, values)


def double_quant(A, col_stats=None, row_stats=None, out_col=None, out_row=None, threshold=0.0):
    """Row- and column-normalised int8 quantisation (ref:functional.py:2517-2604).
    Returns (out_row, out_col, row_stats, col_stats, coo_tensor)."""
    device = A.device
    assert A.dtype == torch.half
    assert device.type == "cuda"
    cols = A.shape[-1]
    rows = A.shape[0] * A.shape[1] if len(A.shape) == 3 else A.shape[0]
    nnz_row_ptr = None
    if row_stats is None or col_stats is None:
        row_stats, col_stats, nnz_row_ptr = get_colrow_absmax(A, threshold=threshold)
    # every element is written by the kernel (outliers as 0), so no zero-fill (the reference's torch.zeros
    # costs two 1-byte-per-element fill passes: ~20 us at 4096 x 11008)
    if out_col is None:
        out_col = torch.empty(A.shape, device=device, dtype=torch.int8)
    if out_row is None:
        out_row = torch.empty(A.shape, device=device, dtype=torch.int8)
    coo_tensor = None
    prev_device = pre_call(A.device)
    is_on_gpu([A, col_stats, row_stats, out_col, out_row])
    if threshold > 0.0 and nnz_row_ptr is not None and nnz_row_ptr[-1].item() > 0:
        nnz = nnz_row_ptr[-1].item()
        coo_tensor = coo_zeros(A.shape[0], A.shape[1], nnz, device)
        lib.cdouble_rowcol_quant(get_ptr(A), get_ptr(row_stats), get_ptr(col_stats), get_ptr(out_col),
                                 get_ptr(out_row), get_ptr(coo_tensor.rowidx), get_ptr(coo_tensor.colidx),
                                 get_ptr(coo_tensor.values), get_ptr(nnz_row_ptr), ct.c_float(threshold),
                                 ct.c_int32(rows), ct.c_int32(cols))
        val, idx = torch.sort(coo_tensor.rowidx)
        coo_tensor.rowidx = val
        coo_tensor.colidx = coo_tensor.colidx[idx]
        coo_tensor.values = coo_tensor.values[idx]
    else:
        lib.cdouble_rowcol_quant(get_ptr(A), get_ptr(row_stats), get_ptr(col_stats), get_ptr(out_col),
                                 get_ptr(out_row), None, None, None, None, ct.c_float(0.0), ct.c_int32(rows),
                                 ct.c_int32(cols))
    post_call(prev_device)
    return out_row, out_col, row_stats, col_stats, coo_tensor


def spmm_coo(cooA: COOSparseTensor, B: Tensor, out: Optional[Tensor] = None) -> Tensor:
    """out = A_coo @ B (fp16), ref:functional.py:2656-2701.  The reference routes this to a cuSPARSE
    SpMM (cspmm_coo, left commented out in its C-ABI, Q18); here: the nonzeros are stably sorted by row,
    row pointers built, and cspmm_coo_rows sums each row's products in fp32 in that order."""
    if out is None:
        out = torch.empty((cooA.rows, B.shape[1]), device=B.device, dtype=B.dtype)
    nnz = cooA.nnz
    assert cooA.rowidx.numel() == nnz and cooA.colidx.numel() == nnz and cooA.values.numel() == nnz
    assert cooA.cols == B.shape[0]
    assert B.dtype == torch.float16 and out.dtype == torch.float16
    transposed_B = not B.is_contiguous()
    ldb = B.stride()[1 if transposed_B else 0]
    ldc = B.shape[1]
    order = torch.sort(cooA.rowidx.long(), stable=True).indices
    rows_sorted = cooA.rowidx[order]
    colidx = cooA.colidx[order].contiguous()
    values = cooA.values[order].contiguous()
    row_ptr = torch.searchsorted(rows_sorted.long(), torch.arange(cooA.rows + 1, device=B.device)).int()
    prev_device = pre_call(B.device)
    is_on_gpu([row_ptr, colidx, values, B, out])
    lib.cspmm_coo_rows(get_ptr(row_ptr), get_ptr(colidx), get_ptr(values), ct.c_int32(cooA.rows),
                       ct.c_int32(B.shape[1]), ct.c_int32(ldb), get_ptr(B), ct.c_int32(ldc), get_ptr(out),
                       ct.c_bool(transposed_B))
    post_call(prev_device)
    return out


def spmm_coo_very_sparse(cooA: COOSparseTensor, B: Tensor, dequant_stats: Optional[Tensor] = None,
                         out: Optional[Tensor] = None) -> Tensor:
    """out += A_coo @ B for <= 32 nonzeros per row, ref:functional.py:2704-2782: one workgroup per nonzero
    row (rows with most nonzeros first), fp16 accumulation; int8 B is dequantised by dequant_stats / 127."""
    if out is None:
        out = torch.zeros((cooA.rows, B.shape[1]), device=B.device, dtype=cooA.values.dtype)
    nnz = cooA.nnz
    prev_device = pre_call(B.device)
    assert cooA.rowidx.numel() == nnz and cooA.colidx.numel() == nnz and cooA.values.numel() == nnz
    assert cooA.cols == B.shape[0], f"{cooA.cols} vs {B.shape}"
    if not B.is_contiguous():
        raise ValueError("spmm_coo_very_sparse: B must be row-major contiguous (the kernel reads B rows)")
    values, counts = torch.unique(cooA.rowidx, return_counts=True)
    offset = counts.cumsum(0).int()
    max_count, max_idx = torch.sort(counts, descending=True, stable=True)
    max_idx = max_idx.int()
    max_count = max_count.int()
    assert max_count[0] <= 32, f"Current max count per row is 8 but found {max_count[0]}."
    assert B.dtype in [torch.float16, torch.int8]
    is_on_gpu([cooA.rowidx, cooA.colidx, cooA.values, B, out, dequant_stats])
    fn = lib.cspmm_coo_very_sparse_naive_fp16 if B.dtype == torch.float16 else lib.cspmm_coo_very_sparse_naive_int8
    fn(get_ptr(max_count), get_ptr(max_idx), get_ptr(offset), get_ptr(cooA.rowidx), get_ptr(cooA.colidx),
       get_ptr(cooA.values), get_ptr(B), get_ptr(out), get_ptr(dequant_stats), ct.c_int32(counts.numel()),
       ct.c_int32(nnz), ct.c_int32(cooA.rows), ct.c_int32(B.shape[1]), ct.c_int32(B.shape[1]))
    post_call(prev_device)
    return out


def int8_row_quant(A: Tensor, out_row: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    """(CA, row_stats) of double_quant(A) with threshold 0 -- the row-normalised int8 matrix and its fp32
    row absmax -- in one pass over A (cint8_row_quant_fp16); what the LLM.int8 forward needs when no
    backward will use CAt.  Falls back to double_quant for shapes the one-pass kernel does not take."""
    assert A.dtype == torch.half and A.device.type == "cuda"
    rows = A.numel() // A.shape[-1]
    cols = A.shape[-1]
    A2 = A if A.is_contiguous() else A.contiguous()
    if out_row is None:
        out_row = torch.empty(A.shape, device=A.device, dtype=torch.int8)
    row_stats = torch.empty((rows,), device=A.device, dtype=torch.float32)
    prev_device = pre_call(A.device)
    is_on_gpu([A2, row_stats, out_row])
    rc = lib.cint8_row_quant_fp16(get_ptr(A2), get_ptr(row_stats), get_ptr(out_row), ct.c_int32(rows), ct.c_int32(cols))
    post_call(prev_device)
    if rc != 0:
        CA, _, SCA, _, _ = double_quant(A2, out_row=out_row)
        return CA, SCA
    return out_row, row_stats


def extract_outliers(A, SA, idx):
    """Gather int8 columns `idx` of a turing/ampere-tiled matrix (ref:functional.py:2914-2936)."""
    shapeA, formatA = SA[0], SA[1]
    assert formatA in ["col_turing", "col_ampere"]
    assert A.device.type == "cuda"
    out = torch.zeros((shapeA[0], idx.numel()), dtype=torch.int8, device=A.device)
    prev_device = pre_call(A.device)
    fn = lib.cextractOutliers_turing if formatA == "col_turing" else lib.cextractOutliers_ampere
    fn(get_ptr(A), get_ptr(idx), get_ptr(out), ct.c_int32(idx.numel()), ct.c_int32(shapeA[0]),
       ct.c_int32(shapeA[1]))
    post_call(prev_device)
    return out


# ----------------------------------------------------------------------------- optimizers
_OPT_NAMES = ("adam", "momentum", "rmsprop", "adagrad", "lion")
# C-ABI names per optimizer and gradient dtype (fp32, fp16, bf16); the 32-bit names keep the
# reference's mixed suffixes (ref:sycl/pythonInterface.cpp:230-241, python functional.py:29-56)
_SUFFIX32 = {"adam": ("fp32", "fp16", "bf16"), "momentum": ("32", "16", "bf16"), "rmsprop": ("32", "16", "bf16"),
             "adagrad": ("32", "16", "bf16"), "lion": ("fp32", "fp16", "bf16")}
_DTYPE_INDEX = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}


def _opt_fn(optimizer_name: str, g: Tensor, blockwise: bool):
    name = "adam" if optimizer_name == "lamb" and not blockwise else optimizer_name
    if name not in _OPT_NAMES or g.dtype not in _DTYPE_INDEX:
        raise ValueError(f"Gradient+optimizer bit data type combination not supported: grad {g.dtype}, "
                         f"optimizer {optimizer_name}")
    i = _DTYPE_INDEX[g.dtype]
    sym = (f"c{name}_8bit_blockwise_grad_{('fp32', 'fp16', 'bf16')[i]}" if blockwise
           else f"c{name}32bit_grad_{_SUFFIX32[name][i]}")
    return getattr(lib, sym)


def optimizer_update_8bit_blockwise(optimizer_name: str, g: Tensor, p: Tensor, state1: Tensor,
                                    state2: Optional[torch.Tensor], beta1: float, beta2: float, eps: float, step: int,
                                    lr: float, qmap1: Tensor, qmap2: Optional[torch.Tensor], absmax1: Tensor,
                                    absmax2: Optional[torch.Tensor], weight_decay: float = 0.0,
                                    gnorm_scale: float = 1.0, skip_zeros=False) -> None:
    """In-place optimizer step with 8-bit states quantised per 2048-element block with the dynamic
    maps (ref:functional.py:1754-1814 -> c<name>_8bit_blockwise_grad_<T>)."""
    if state1.dtype != torch.uint8:
        raise ValueError(f"Gradient+optimizer bit data type combination not supported: grad {g.dtype}, "
                         f"optimizer {state1.dtype}")
    optim_func = _opt_fn(optimizer_name, g, True)
    is_on_gpu([p, g, state1, state2, qmap1, qmap2, absmax1, absmax2])
    prev_device = pre_call(g.device)
    optim_func(get_ptr(p), get_ptr(g), get_ptr(state1), get_ptr(state2), ct.c_float(beta1), ct.c_float(beta2),
               ct.c_float(eps), ct.c_int32(step), ct.c_float(lr), get_ptr(qmap1), get_ptr(qmap2), get_ptr(absmax1),
               get_ptr(absmax2), ct.c_float(weight_decay), ct.c_float(gnorm_scale), ct.c_bool(skip_zeros),
               ct.c_int32(g.numel()))
    post_call(prev_device)


def optimizer_update_32bit(optimizer_name: str, g: Tensor, p: Tensor, state1: Tensor, beta1: float, eps: float,
                           step: int, lr: float, state2: Optional[torch.Tensor] = None, beta2: float = 0.0,
                           weight_decay: float = 0.0, gnorm_scale: float = 1.0,
                           unorm_vec: Optional[torch.Tensor] = None, max_unorm: float = 0.0,
                           skip_zeros=False) -> None:
    """In-place optimizer step with fp32 states (ref:functional.py:1526-1615 -> c<name>32bit_grad_<T>).
    max_unorm > 0 (update-norm clipping, kPreconditionOptimizer32bit) is not supported here."""
    if max_unorm > 0.0:
        raise NotImplementedError("max_unorm > 0 is not supported by the MI355X backend")
    optim_func = _opt_fn(optimizer_name, g, False)
    param_norm = 0.0
    is_on_gpu([g, p, state1, state2, unorm_vec])
    prev_device = pre_call(g.device)
    optim_func(get_ptr(g), get_ptr(p), get_ptr(state1), get_ptr(state2), get_ptr(unorm_vec), ct.c_float(max_unorm),
               ct.c_float(param_norm), ct.c_float(beta1), ct.c_float(beta2), ct.c_float(eps),
               ct.c_float(weight_decay), ct.c_int32(step), ct.c_float(lr), ct.c_float(gnorm_scale),
               ct.c_bool(skip_zeros), ct.c_int32(g.numel()))
    post_call(prev_device)
