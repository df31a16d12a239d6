"""Shared helpers for the parity tests (numpy <-> torch, incl. bf16 bit patterns)."""
import numpy as np
import torch

from oracle import ref

DTYPES = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}


def to_torch(a: np.ndarray, kind: str, device) -> torch.Tensor:
    """kind: 'fp32'|'fp16'|'bf16' (bf16 given as uint16 bits) or a raw numpy dtype."""
    if kind == "bf16":
        return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).view(torch.bfloat16).to(device)
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


def to_numpy(t: torch.Tensor, kind: str) -> np.ndarray:
    t = t.detach().cpu().contiguous()
    if kind == "bf16":
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def same_bits(a: np.ndarray, b: np.ndarray) -> bool:
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    return a.shape == b.shape and a.tobytes() == b.tobytes()


def f32_of(a: np.ndarray, kind: str) -> np.ndarray:
    return ref.as_f32(a, kind)
