"""QuantState packing helpers (ref:python_src_quants/utils.py:169-204)."""
from __future__ import annotations

import json

import torch


def pack_dict_to_tensor(source_dict):
    """dict -> JSON -> uint8 tensor (the `quant_state.bitsandbytes__*` state-dict entry)."""
    return torch.tensor(list(json.dumps(source_dict).encode("utf-8")), dtype=torch.uint8)


def unpack_tensor_to_dict(tensor_data):
    return json.loads(bytes(tensor_data.cpu().numpy()).decode("utf-8"))


LINEAR_8BIT_WEIGHTS_FORMAT_MAPPING = {"row": 0, "col32": 1, "col_turing": 2, "col_ampere": 3}
INVERSE_LINEAR_8BIT_WEIGHTS_FORMAT_MAPPING = {v: k for k, v in LINEAR_8BIT_WEIGHTS_FORMAT_MAPPING.items()}
