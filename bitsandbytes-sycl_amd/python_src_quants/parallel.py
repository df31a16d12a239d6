"""Output-feature (column) sharding of 4-bit linears across the GPUs of one node.

Not in the reference (it has no multi-GPU code); this is the MI355X scale-out
of the hot path the north star asks for: W [N, K] is split by output features (rows of W),
rank r owns rows [r*N/g, (r+1)*N/g) — its packed bytes, absmax and (re-quantised) nested
statistics are independent because NF4 blocks never straddle rows when K % blocksize == 0
(absmax index = (n*K + k) / bs).  Activations are replicated; each rank computes its
[M, N/g] slice with the fused NF4 GEMM (or the GEMV at M == 1) and one RCCL all-gather over
xGMI assembles [g, M, N/g] (bf16), viewed as [M, N] by `gathered_to_rows`.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist

from . import functional as F


def shard_range(n_out: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous output-feature range of `rank` (world must divide n_out)."""
    if n_out % world:
        raise ValueError(f"out_features {n_out} not divisible by world size {world}")
    per = n_out // world
    return rank * per, (rank + 1) * per


def shard_packed_rows(packed: torch.Tensor, absmax: torch.Tensor, shape, blocksize: int, start: int, end: int):
    """Slice a non-nested 4-bit quantised weight [N, K] (packed uint8 [(N*K+1)//2, 1], fp32 absmax) to
    rows [start, end).  Requires K % blocksize == 0 and K even so rows own whole bytes and blocks."""
    N, K = shape
    if K % blocksize or K % 2:
        raise ValueError("row sharding needs K % blocksize == 0 and even K")
    flat = packed.reshape(-1)
    p = flat[start * K // 2:end * K // 2].reshape(-1, 1)
    a = absmax[start * K // blocksize:end * K // blocksize]
    return p, a


def gather_columns(y_local: torch.Tensor, world: int, group=None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """All-gather the per-rank [M, n] slices into [world, M, n] (one collective; RCCL on GPU)."""
    if world == 1:
        return y_local.unsqueeze(0)
    y_local = y_local.contiguous()
    if out is None:
        out = torch.empty((world,) + tuple(y_local.shape), dtype=y_local.dtype, device=y_local.device)
    if dist.get_backend(group) == "gloo":
        dist.all_gather(list(out.unbind(0)), y_local, group=group)
    else:
        dist.all_gather_into_tensor(out, y_local, group=group)
    return out


def _gather_async(out: torch.Tensor, y: torch.Tensor, group=None):
    """Start the all-gather of y [Mc, n] into out [world, Mc, n]; returns the work handle."""
    if dist.get_backend(group) == "gloo":
        return dist.all_gather(list(out.unbind(0)), y, group=group, async_op=True)
    return dist.all_gather_into_tensor(out, y, group=group, async_op=True)


def sharded_forward_overlapped(x2: torch.Tensor, local_mm: Callable, world: int, group=None, chunks: int = 2,
                               out: Optional[torch.Tensor] = None, y: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Token-row-chunked sharded forward: the local GEMM of chunk c+1 runs while the all-gather of
    chunk c is in flight (RCCL runs on its own stream; async_op handles order it after the GEMM that
    produced the chunk and before the caller's next use).  local_mm(x_chunk, y_chunk_or_None) returns
    this rank's [Mc, n] slice.  Returns [chunks, world, Mc, n] (chunk c = token rows c*Mc .. +Mc);
    `chunked_to_rows` assembles [M, world*n].  chunks must divide M (else a single chunk is used)."""
    M = x2.shape[0]
    if chunks < 1 or M % chunks:
        chunks = 1
    Mc = M // chunks
    works = []
    for c in range(chunks):
        rows = slice(c * Mc, (c + 1) * Mc)
        yc = local_mm(x2[rows], None if y is None else y[rows])
        if out is None:
            out = torch.empty((chunks, world, Mc, yc.shape[1]), dtype=yc.dtype, device=yc.device)
        if world == 1:
            out[c, 0].copy_(yc)
        else:
            works.append(_gather_async(out[c], yc.contiguous(), group))
    for w in works:
        w.wait()
    return out


def chunked_to_rows(g: torch.Tensor) -> torch.Tensor:
    """[chunks, world, Mc, n] -> [chunks*Mc, world*n] (a copy)."""
    c, w, mc, n = g.shape
    return g.permute(0, 2, 1, 3).reshape(c * mc, w * n)


def gathered_to_rows(g: torch.Tensor) -> torch.Tensor:
    """[world, M, n] -> [M, world*n] (a copy; consumers that can index [world, M, n] should not call this)."""
    w, m, n = g.shape
    return g.permute(1, 0, 2).reshape(m, w * n)


class ColumnShardedLinear4bit(torch.nn.Module):
    """Holds this rank's NF4/FP4 shard of a linear layer's weight and runs the sharded forward."""

    def __init__(self, weight: torch.Tensor, world: int, rank: int, group=None, quant_type: str = "nf4",
                 blocksize: int = 64, compress_statistics: bool = True, device=None):
        super().__init__()
        n_out, k_in = weight.shape
        self.world, self.rank, self.group = world, rank, group
        self.start, self.end = shard_range(n_out, world, rank)
        device = device or torch.device("cuda", torch.cuda.current_device())
        w = weight[self.start:self.end].to(device)
        self.qweight, self.quant_state = F.quantize_4bit(w, blocksize=blocksize, quant_type=quant_type,
                                                         compress_statistics=compress_statistics)
        self.out_features, self.in_features = n_out, k_in

    def forward_local(self, x: torch.Tensor) -> torch.Tensor:
        x2 = x.reshape(-1, self.in_features)
        if x2.shape[0] == 1:
            return F.gemv_4bit(x2, self.qweight.t(), state=self.quant_state)
        return F.gemm_4bit(x2, self.qweight, self.quant_state)

    def forward(self, x: torch.Tensor, assemble: bool = True, chunks: int = 1) -> torch.Tensor:
        """chunks > 1 overlaps the all-gather of each token-row chunk with the next chunk's GEMM
        (result layout [chunks, world, M/chunks, n] when assemble=False)."""
        if chunks > 1:
            x2 = x.reshape(-1, self.in_features)

            first = [True]

            def mm(xc, yc):   # one dequantisation of the shard per forward on the library path
                r = F.gemm_4bit(xc, self.qweight, self.quant_state, out=yc, reuse_weight=not first[0])
                first[0] = False
                return r
            g = sharded_forward_overlapped(x2, mm, self.world, self.group, chunks)
            return chunked_to_rows(g) if assemble else g
        g = gather_columns(self.forward_local(x), self.world, self.group)
        return gathered_to_rows(g) if assemble else g
