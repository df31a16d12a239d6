"""ctypes loader for the gfx950 C-ABI library (replaces ref:python_src_quants/cextension.py:43-129).

The library is built in-tree (``bitsandbytes-sycl_amd/csrc`` -> ``libbitsandbytes_hip.so``
next to this file).  There is no CPU fallback: if the library is missing, ``lib`` is a
stub whose every attribute access raises, so GPU ops fail loudly instead of silently
running something else.
"""
from __future__ import annotations

import ctypes as ct
import logging
import os
from pathlib import Path

logger = logging.getLogger(__name__)

PACKAGE_DIR = Path(__file__).parent
LIBRARY_NAME = "libbitsandbytes_hip.so"


def get_hip_bnb_library_path() -> Path:
    override = os.environ.get("BNB_HIP_LIBRARY")
    return Path(override) if override else PACKAGE_DIR / LIBRARY_NAME


class BNBNativeLibrary:
    _lib: ct.CDLL
    compiled_with_hip = True

    def __init__(self, lib: ct.CDLL):
        self._lib = lib
        # restypes the reference sets at load (cextension.py:82-84) + the additive entry points
        lib.get_context.restype = ct.c_void_p
        lib.get_cusparse.restype = ct.c_void_p
        lib.cget_managed_ptr.restype = ct.c_void_p
        lib.cget_stream.restype = ct.c_void_p
        lib.cget_last_error_message.restype = ct.c_char_p
        lib.cgemm_4bit_workspace_bytes.restype = ct.c_longlong
        lib.cigemmlt_workspace_bytes.restype = ct.c_longlong
        lib.chgemm_tn_workspace_bytes.restype = ct.c_longlong
        lib.cipc_allgather_buffer_bytes.restype = ct.c_longlong
        lib.cipc_alloc.restype = ct.c_void_p
        lib.cipc_alloc.argtypes = [ct.c_longlong, ct.POINTER(ct.c_int)]
        for name in ("cigemmlt_turing_32", "cigemmlt_turing_8", "cigemmlt_turing_8_rowscale",
                     "cigemmlt_ampere_32", "cigemmlt_ampere_8", "cigemmlt_ampere_8_rowscale",
                     "cigemmlt_row_dequant_fp16", "cigemm_row_i32", "cigemmlt_row_dequant_ws_fp16",
                     "cigemm_row_i32_ws", "cgemm_tn_bf16", "cgemm_tn_fp16", "cgemm_tn_set_search", "cgemm_tn_plan",
                     "chgemm_tn_bf16", "chgemm_tn_fp16", "cprobe_mfma", "cprobe_hbm_read",
                     "cget_last_error", "cget_abi_version",
                     "cgemm_4bit_inference_naive_nested_fp16", "cgemm_4bit_inference_naive_nested_bf16",
                     "cdequantize_blockwise_nested_fp16_fp4", "cdequantize_blockwise_nested_fp16_nf4",
                     "cdequantize_blockwise_nested_bf16_fp4", "cdequantize_blockwise_nested_bf16_nf4",
                     "cint8_row_quant_fp16", "cgemm_4bit_inference_nested_ws_bf16",
                     "cgemm_4bit_inference_nested_ws_fp16", "cset_cpu_threads", "cgemm_4bit_fewtok_takes", "chgemm_tn_ws_bf16", "chgemm_tn_ws_fp16",
                     "cipc_handle_size", "cipc_get_handle", "cipc_open_handle", "cipc_close_handle", "callgather_ipc_16",
                     "cprobe_lds_poison", "cprobe_lds_peek", "croctx_enabled"):
            getattr(lib, name).restype = ct.c_int

    def __getattr__(self, item):
        fn = getattr(self._lib, item)
        setattr(self, item, fn)          # later lookups hit the instance dict
        return fn


class _MissingLibrary:
    def __init__(self, err: Exception):
        self._err = err

    def __getattr__(self, item):
        raise RuntimeError(
            f"bitsandbytes HIP library not loaded ({self._err}); build it with "
            f"`make -C bitsandbytes-sycl_amd/csrc` (gfx950). There is no CPU fallback."
        )

    def __bool__(self):
        return False


def get_native_library():
    path = get_hip_bnb_library_path()
    dll = ct.cdll.LoadLibrary(str(path))
    if not hasattr(dll, "get_context"):
        raise RuntimeError(f"{path} does not export the bitsandbytes C-ABI")
    return BNBNativeLibrary(dll)


try:
    lib = get_native_library()
    HIP_AVAILABLE = True
except Exception as e:  # noqa: BLE001 - reported loudly on first use
    lib = _MissingLibrary(e)
    HIP_AVAILABLE = False
    logger.error("Could not load the bitsandbytes HIP library: %s", e)
