"""Quantisation maps used as *inputs* by the hot path (TEST INFRASTRUCTURE ONLY).

The reference builds its 256-entry dynamic code with torch float32 ops
(ref:python_src_quants/functional.py:339-391).  The exact float32 values depend
on torch.linspace's algorithm, so this restatement calls the same torch
functions in the same order; the result is fed to the kernels as data.
"""
from __future__ import annotations

import numpy as np
import torch


def create_dynamic_map(signed: bool = True, max_exponent_bits: int = 7, total_bits: int = 8) -> np.ndarray:
    """Dynamic (exponent + fraction) 8-bit map, functional.py:339-391 restated."""
    data = []
    non_sign_bits = total_bits - 1
    additional_items = 2 ** (non_sign_bits - max_exponent_bits) - 1
    for i in range(max_exponent_bits):
        if signed:
            fraction_items = int(2 ** (i + non_sign_bits - max_exponent_bits) + 1)
        else:
            fraction_items = int(2 ** (i + non_sign_bits - max_exponent_bits + 1) + 1)
        bounds = torch.linspace(0.1, 1, fraction_items)
        means = (bounds[:-1] + bounds[1:]) / 2.0
        scale = 10 ** (-(max_exponent_bits - 1) + i)
        data += (scale * means).tolist()
        if signed:
            data += (-scale * means).tolist()
    if additional_items > 0:
        bounds = torch.linspace(0.1, 1, additional_items + 1)
        means = (bounds[:-1] + bounds[1:]) / 2.0
        scale = 10 ** (-(max_exponent_bits - 1) + max_exponent_bits - 1)
        data += (scale * means).tolist()
        if signed:
            data += (-scale * means).tolist()
    data.append(0)
    data.append(1.0)
    assert len(data) == 2 ** total_bits
    data += [0] * (256 - len(data))
    data.sort()
    return torch.tensor(data, dtype=torch.float32).numpy()


def nf4_padded_256() -> np.ndarray:
    """Config-1 CPU form: the 16 NF4 values padded to a 256-entry code."""
    from .ref import NF4_TREE_VALUES
    code = np.zeros(256, dtype=np.float32)
    code[:16] = NF4_TREE_VALUES
    return code
