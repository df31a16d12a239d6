"""MI355X (gfx950) backend for the bitsandbytes quantized-matmul hot path.

Drop-in for ref:python_src_quants/__init__.py on the hot path: `functional`, `nn`,
`matmul` (LLM.int8) and `matmul_4bit` (NF4/FP4), backed by the HIP C-ABI library
`libbitsandbytes_hip.so` built from ../csrc.
"""
from . import functional, nn, optim, utils
from .autograd._functions import MatmulLtState, MatMul4Bit, MatMul8bitLt, matmul, matmul_4bit
from .cextension import HIP_AVAILABLE, lib

__version__ = "0.43.2.mi355x0"

__all__ = ["functional", "nn", "optim", "utils", "matmul", "matmul_4bit", "MatmulLtState", "MatMul4Bit", "MatMul8bitLt",
           "lib", "HIP_AVAILABLE"]
