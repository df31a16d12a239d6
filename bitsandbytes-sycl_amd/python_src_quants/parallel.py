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


def shard_quantized_4bit(packed: torch.Tensor, state: "F.QuantState", world: int, rank: int):
    """Rank `rank`'s output-feature shard of an already quantised 4-bit weight [N, K] (e.g. a Linear4bit or an
    NF4 checkpoint restored by Params4bit.from_prequantized, ref:nn/modules.py:271-289), without the float weight.

    Returns (packed_shard [(n*K)//2, 1] uint8, QuantState with shape (n, K)).  The packed bytes and the first-level
    block statistics are sliced (K % blocksize == 0: no block straddles two rows).  Compressed (nested) statistics,
    the Linear4bit default (ref:nn/modules.py:385; layout ref:functional.py:1243-1257), are handled two ways:
      * the shard starts on a second-level block (its first block index is a multiple of the nested blocksize,
        true for every Llama-2-70B projection at 8 ranks): the uint8 codes and their fp32 second-level scales are
        sliced too, with the full weight's offset -- the shard decodes to exactly the full weight's block scales;
      * otherwise the shard's fp32 block scales are decoded and re-compressed for the shard alone (offset = their
        mean, dynamic 8-bit map, the nested blocksize) -- what quantize_4bit would store for these rows."""
    N, K = state.shape
    bs = state.blocksize
    if K % bs or K % 2:
        raise ValueError("row sharding needs K % blocksize == 0 and even K")
    start, end = shard_range(N, world, rank)
    n = end - start
    b0, b1 = start * K // bs, end * K // bs
    flat = packed.reshape(-1)
    p = flat[start * K // 2:end * K // 2].reshape(-1, 1)
    shape = torch.Size([n, K])
    if not state.nested:
        return p, F.QuantState(absmax=state.absmax[b0:b1], shape=shape, code=state.code, blocksize=bs,
                               quant_type=state.quant_type, dtype=state.dtype)
    s2 = state.state2
    bs2 = s2.blocksize
    if b0 % bs2 == 0:
        e2 = (b1 + bs2 - 1) // bs2
        state2 = F.QuantState(absmax=s2.absmax[b0 // bs2:e2], blocksize=bs2, code=s2.code, dtype=s2.dtype)
        return p, F.QuantState(absmax=state.absmax[b0:b1], shape=shape, code=state.code, blocksize=bs,
                               quant_type=state.quant_type, dtype=state.dtype, offset=state.offset, state2=state2)
    absmax = F._absmax_fp32(state)[b0:b1].contiguous()
    offset = absmax.mean()
    qabsmax, state2 = F.quantize_blockwise(absmax - offset, blocksize=bs2)
    return p, F.QuantState(absmax=qabsmax, shape=shape, code=state.code, blocksize=bs, quant_type=state.quant_type,
                           dtype=state.dtype, offset=offset, state2=state2)


def fuse_quantized_4bit(parts):
    """Concatenate already quantised 4-bit weights [n_i, K] along the output features into ONE weight
    [sum n_i, K] -- the inverse of shard_quantized_4bit, for projections that read the same input (a decoder
    layer's q/k/v, or gate/up): one GEMV / GEMM launch then streams all of them (round 3, bench
    `llama2_70b_rank_shard_config5.decode_fused`).  `parts` is a list of (packed, QuantState) with equal K,
    blocksize, quant_type, code and dtype.  Returns (packed [(N*K)//2, 1] uint8, QuantState with shape (N, K)) and the
    output column offsets [0, n_0, n_0 + n_1, ...] (split the result with split_fused_columns).

    Packed bytes and first-level statistics concatenate exactly (K % blocksize == 0: no block straddles two rows).
    Compressed (nested) statistics are decoded and re-compressed for the fused weight (offset = their mean, dynamic
    8-bit map, the nested blocksize) -- what quantize_4bit stores for the concatenated rows; each part's offset is
    its own mean, so the codes of the parts alone cannot simply be concatenated."""
    if not parts:
        raise ValueError("fuse_quantized_4bit: no parts")
    K = parts[0][1].shape[1]
    st0 = parts[0][1]
    for _, st in parts:
        if (st.shape[1] != K or st.blocksize != st0.blocksize or st.quant_type != st0.quant_type
                or st.dtype != st0.dtype or bool(st.nested) != bool(st0.nested)
                or not torch.equal(st.code, st0.code)):
            raise ValueError("fuse_quantized_4bit: parts need equal K, blocksize, quant_type, code, dtype and "
                             "statistics format")
    if K % st0.blocksize or K % 2:
        raise ValueError("fuse_quantized_4bit needs K % blocksize == 0 and even K")
    packed = torch.cat([p.reshape(-1) for p, _ in parts]).reshape(-1, 1)
    N = sum(st.shape[0] for _, st in parts)
    offsets = [0]
    for _, st in parts:
        offsets.append(offsets[-1] + st.shape[0])
    shape = torch.Size([N, K])
    if not st0.nested:
        absmax = torch.cat([st.absmax for _, st in parts])
        return packed, F.QuantState(absmax=absmax, shape=shape, code=st0.code, blocksize=st0.blocksize,
                                    quant_type=st0.quant_type, dtype=st0.dtype), offsets
    absmax = torch.cat([F._absmax_fp32(st) for _, st in parts]).contiguous()
    offset = absmax.mean()
    qabsmax, state2 = F.quantize_blockwise(absmax - offset, blocksize=st0.state2.blocksize)
    return packed, F.QuantState(absmax=qabsmax, shape=shape, code=st0.code, blocksize=st0.blocksize,
                                quant_type=st0.quant_type, dtype=st0.dtype, offset=offset, state2=state2), offsets


def split_fused_columns(y: torch.Tensor, offsets):
    """Views of the fused output's column ranges (fuse_quantized_4bit offsets), one per original projection."""
    return [y[..., a:b] for a, b in zip(offsets[:-1], offsets[1:])]


def shard_int8_rows(CB: torch.Tensor, SCB: torch.Tensor, world: int, rank: int):
    """Rank `rank`'s output-feature shard of an LLM.int8 weight: the rows of CB (int8 [N, K], row-normalised) and
    of its row statistics SCB (fp32 [N]) -- Int8Params' state (ref:nn/modules.py:559-632).  Rows quantise
    independently, so the slice is exactly what double_quant gives for those rows."""
    start, end = shard_range(CB.shape[0], world, rank)
    return CB[start:end], SCB[start:end]


# At world 1 the gathers below are skipped (the slice IS the output).  set_force_collective(True) runs them anyway
# through the initialised process group -- so a one-GPU box exercises the RCCL all-gather, its async overlap and its
# HIP-graph capture exactly as the multi-GPU step does (tests/test_rccl_gpu.py).
_FORCE_COLLECTIVE = [False]


def set_force_collective(on: bool) -> None:
    """Run the all-gathers even at world size 1 (needs an initialised process group); test / rehearsal knob."""
    _FORCE_COLLECTIVE[0] = bool(on)


def _collective(world: int) -> bool:
    return world > 1 or (_FORCE_COLLECTIVE[0] and dist.is_available() and dist.is_initialized())


def gather_columns(y_local: torch.Tensor, world: int, group=None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """All-gather the per-rank [M, n] slices into [world, M, n] (one collective; RCCL on GPU)."""
    if not _collective(world):
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
                               out: Optional[torch.Tensor] = None, y: Optional[torch.Tensor] = None,
                               rows_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Token-row-chunked sharded forward: the local GEMM of chunk c+1 runs while the all-gather of
    chunk c is in flight (RCCL runs on its own stream; async_op handles order it after the GEMM that
    produced the chunk and before the caller's next use).  local_mm(x_chunk, y_chunk_or_None) returns
    this rank's [Mc, n] slice.  Returns [chunks, world, Mc, n] (chunk c = token rows c*Mc .. +Mc);
    `chunked_to_rows` assembles [M, world*n].  chunks must divide M (else a single chunk is used).
    rows_out ([M, world*n]): assemble there as well, chunk by chunk as each gather lands, so chunk c's
    copy overlaps chunk c+1's gather; returns rows_out then."""
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
        if not _collective(world):
            out[c, 0].copy_(yc)
        else:
            works.append(_gather_async(out[c], yc.contiguous(), group))
    for c, w in enumerate(works):
        w.wait()
        if rows_out is not None:
            rows_out[c * Mc:(c + 1) * Mc].view(Mc, world, -1).copy_(out[c].permute(1, 0, 2))
    if rows_out is not None:
        if not works:
            rows_out.copy_(out.reshape(rows_out.shape))
        return rows_out
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

    def __init__(self, weight: Optional[torch.Tensor], world: int, rank: int, group=None, quant_type: str = "nf4",
                 blocksize: int = 64, compress_statistics: bool = True, device=None):
        super().__init__()
        self.world, self.rank, self.group = world, rank, group
        if weight is None:      # filled by from_quantized
            return
        n_out, k_in = weight.shape
        self.start, self.end = shard_range(n_out, world, rank)
        device = device or torch.device("cuda", torch.cuda.current_device())
        w = weight[self.start:self.end].to(device)
        self.qweight, self.quant_state = F.quantize_4bit(w, blocksize=blocksize, quant_type=quant_type,
                                                         compress_statistics=compress_statistics)
        self.out_features, self.in_features = n_out, k_in

    @classmethod
    def from_quantized(cls, packed: torch.Tensor, state: "F.QuantState", world: int, rank: int, group=None,
                       device=None) -> "ColumnShardedLinear4bit":
        """This rank's shard of an already quantised weight (a Linear4bit's packed bytes + QuantState, or a
        pre-quantised checkpoint), sliced by shard_quantized_4bit -- no float weight is needed on any rank."""
        self = cls(None, world, rank, group)
        n_out, k_in = state.shape
        self.start, self.end = shard_range(n_out, world, rank)
        p, st = shard_quantized_4bit(packed, state, world, rank)
        if device is not None:
            p = p.to(device)
            st.to(device)
            st.code = st.code.to(device)
        self.qweight, self.quant_state = p, st
        self.out_features, self.in_features = n_out, k_in
        return self

    def forward_local(self, x: torch.Tensor) -> torch.Tensor:
        x2 = x.reshape(-1, self.in_features)
        if x2.shape[0] == 1:
            return F.gemv_4bit(x2, self.qweight.t(), state=self.quant_state)
        return F.gemm_4bit(x2, self.qweight, self.quant_state)

    def decode_step(self, dtype=torch.bfloat16, gather: str = "rccl") -> ShardedDecode:
        """A static-buffer M = 1 step (this shard's GEMV + one all-gather) for graph capture: ShardedDecode.
        gather="ipc": the one-shot peer-memory all-gather (IpcAllGather) instead of RCCL."""
        fn = lambda x, y: F.gemv_4bit(x, self.qweight.t(), out=y, state=self.quant_state)  # noqa: E731
        return ShardedDecode(fn, self.in_features, self.end - self.start, self.world, self.group, dtype,
                             self.qweight.device, gather=gather, rank=self.rank)

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
            if not assemble:
                return sharded_forward_overlapped(x2, mm, self.world, self.group, chunks)
            rows = torch.empty((x2.shape[0], self.out_features), dtype=x2.dtype, device=x2.device)
            return sharded_forward_overlapped(x2, mm, self.world, self.group, chunks, rows_out=rows)
        g = gather_columns(self.forward_local(x), self.world, self.group)
        return gathered_to_rows(g) if assemble else g


class IpcAllGather:
    """One-shot all-gather of a decode step's [1, n] shard outputs over peer memory (csrc/ipc.hip, C-ABI
    callgather_ipc_16): SURVEY §8(e) -- at M = 1 the gather moves KB and RCCL's ~10-20 us latency would dominate a
    decode layer, so each rank pushes its slice straight into every peer's exchange buffer (opened once through
    hipIpc handles exchanged over the process group) with an epoch flag, waits (bounded) for all peers' flags and
    copies the assembled [1, world * n] row out -- ONE kernel, no host synchronisation, HIP-graph capturable.  RCCL stays
    the prefill all-gather.  The exchange buffers live as long as this object; close() frees them after a barrier.

    Layout of the assembled row: rank j's columns at [j * n, (j + 1) * n) -- gathered_to_rows of the RCCL path.
    Memory: every rank's exchange buffer is uncached or fine-grained device memory, and all ranks must hold the same
    kind (setup raises otherwise -- coarse-grained memory would let the owner's L2 serve stale slots).
    Failure is fail-stop: a step whose wait for a peer timed out writes a NaN row (never the stale slots), and so does
    every later step of this exchange; timeouts() is the sticky count of polls that gave up (0 while healthy) and
    check() raises when it is non-zero."""

    def __init__(self, n_local: int, world: int, rank: int, group=None, device=None, dtype=torch.bfloat16):
        import ctypes as ct
        if dtype not in (torch.bfloat16, torch.float16):
            raise ValueError("IpcAllGather: bf16 / fp16 shards only")
        if n_local % 8:
            raise ValueError("IpcAllGather: the shard width must be a multiple of 8 (whole 16-B pieces)")
        self.n, self.world, self.rank, self.group, self.dtype = n_local, world, rank, group, dtype
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        lib = F.lib
        self._lib = lib
        self._own = None
        self._opened = []
        self.memory_kind = None
        # Every rank takes part in every collective below whatever happened locally (a failing rank sends None / 0),
        # and all ranks raise together: a setup error on one rank must not leave the others waiting in a collective.
        err = None
        with torch.cuda.device(self.device):
            nbytes = int(lib.cipc_allgather_buffer_bytes(world, n_local, 2))
            kind = ct.c_int(-1)
            ptr = lib.cipc_alloc(ct.c_longlong(nbytes), ct.byref(kind))
            handle = None
            if not ptr:
                err = f"cipc_alloc: {lib.cget_last_error_message().decode()}"
            else:
                self._own, self.memory_kind = ptr, {2: "uncached", 1: "fine-grained", 0: "plain"}.get(kind.value)
                h = ct.create_string_buffer(int(lib.cipc_handle_size()))
                if lib.cipc_get_handle(ct.c_void_p(ptr), h):
                    err = f"cipc_get_handle: {lib.cget_last_error_message().decode()}"
                else:
                    handle = h.raw
            handles = [None] * world
            dist.all_gather_object(handles, handle, group=group)
            ptrs = []
            if err is None and all(x is not None for x in handles):
                for j in range(world):
                    if j == rank:
                        ptrs.append(ptr)
                        continue
                    out = ct.c_void_p()
                    if lib.cipc_open_handle(ct.create_string_buffer(handles[j], len(handles[j])), ct.byref(out)):
                        err = f"cipc_open_handle (rank {j}): {lib.cget_last_error_message().decode()}"
                        break
                    ptrs.append(out.value)
                    self._opened.append(out.value)
            elif err is None:
                err = "a peer could not export its exchange buffer"
            oks = [None] * world
            dist.all_gather_object(oks, (err is None, self.memory_kind), group=group)
            kinds = {k for _, k in oks}
            if err is None and all(ok for ok, _ in oks) and (len(kinds) != 1 or
                                                             not kinds <= {"uncached", "fine-grained"}):
                err = f"exchange buffers of different / unsupported memory kinds across ranks: {[k for _, k in oks]}"
            if err is not None or not all(ok for ok, _ in oks):
                self.close(barrier=False)
                raise RuntimeError(f"IpcAllGather setup failed: {err or 'on a peer rank'}")
            self.table = torch.tensor(ptrs, dtype=torch.int64, device=self.device)
            self.state = torch.zeros(4, dtype=torch.int32, device=self.device)
            torch.cuda.synchronize(self.device)
        dist.barrier(group=group)         # every rank has opened every buffer before anyone pushes

    def __call__(self, y: torch.Tensor, rows: torch.Tensor) -> torch.Tensor:
        """Gather y [1, n] (this rank's shard) into rows [1, world * n] on the current stream."""
        if y.dtype != self.dtype or rows.dtype != self.dtype or y.numel() != self.n or rows.numel() != self.n * self.world:
            raise ValueError("IpcAllGather: shard / row buffers do not match the exchange")
        prev = F.pre_call(y.device)
        rc = self._lib.callgather_ipc_16(F.get_ptr(self.table), self.rank, self.world, self.n, F.get_ptr(y),
                                         F.get_ptr(rows), F.get_ptr(self.state))
        F.post_call(prev)
        if rc:
            raise RuntimeError(f"IpcAllGather: callgather_ipc_16 returned {rc}")
        return rows

    def timeouts(self) -> int:
        """Polls that gave up so far (sticky; synchronises with the device).  Non-zero: this rank's rows have been NaN
        since the step that timed out."""
        return int(self.state[1].item())

    def check(self):
        """Raise when any step of this exchange timed out (its rows, and every later step's, are NaN).  Local: a rank can
        raise here while a peer that finished cleanly carries on -- between ranks use check_all()."""
        n = self.timeouts()
        if n:
            raise RuntimeError(f"IpcAllGather: {n} peer wait(s) timed out (last source rank "
                               f"{int(self.state[2].item()) - 1}); the gathered rows are poisoned (NaN)")

    def check_all(self):
        """check() agreed over the group (a collective: every rank must call it): timeouts are asymmetric -- rank A can
        give up on a slow peer B while B later finds A's flag and finishes cleanly -- so the ranks' counts are reduced
        (MAX) first and then every rank raises, or none does (a lone raise left the healthy ranks waiting in
        the next collective until the process-group timeout)."""
        n = self.timeouts()
        dev = torch.device("cpu") if dist.get_backend(self.group) == "gloo" else self.device
        t = torch.tensor([n], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        if int(t.item()):
            raise RuntimeError(f"IpcAllGather: peer wait(s) timed out on {'this rank' if n else 'a peer rank'} "
                               f"(max {int(t.item())} per rank); the gathered rows are poisoned (NaN)")

    def close(self, barrier: bool = True):
        """Unmap the peers' buffers and free this rank's, after every rank stopped pushing (a barrier)."""
        if barrier:
            torch.cuda.synchronize(self.device)
            dist.barrier(group=self.group)
        for p in self._opened:
            self._lib.cipc_close_handle(__import__("ctypes").c_void_p(p))
        self._opened = []
        if barrier:
            dist.barrier(group=self.group)
        if self._own:
            self._lib.cipc_free(__import__("ctypes").c_void_p(self._own))
            self._own = None


class ShardedDecode:
    """The M = 1 (decode) forward of a column-sharded layer on static buffers, so one decode step -- this rank's GEMV
    into `y` [1, n], ONE all-gather of the KB-sized shard outputs into `gathered` [world, 1, n] and the [1, world*n]
    row assembled in `rows` -- can be captured in a HIP graph and replayed (at M = 1 the all-gather is
    latency-bound; replaying the captured step removes the host launch cost of the GEMV, the collective and the copy,
    which is most of a decode step's time at these sizes).  `local_fn(x, y)` writes this rank's [1, n] slice of x
    [1, K] into y (ColumnShardedLinear4bit.decode_step passes the GEMV); the input goes through `set_input`."""

    def __init__(self, local_fn: Callable, in_features: int, n_local: int, world: int, group=None,
                 dtype=torch.bfloat16, device=None, gather: str = "rccl", rank: Optional[int] = None,
                 checked: bool = False):
        # checked (gather="ipc"): every step / replay is followed by IpcAllGather.check() -- a host synchronisation per
        # token that turns a timed-out peer into an exception on the step that hit it (default: check() on demand, and
        # always after capture()'s warm-up and capture)
        self.local_fn, self.world, self.group, self.checked = local_fn, world, group, checked
        self.x = torch.zeros(1, in_features, dtype=dtype, device=device)
        self.gathered = torch.empty(world, 1, n_local, dtype=dtype, device=device)
        self.graph = None
        # gather="ipc": the one-shot peer-memory all-gather (IpcAllGather) instead of RCCL's all_gather_into_tensor
        self.ipc = None
        if gather == "ipc":
            r = dist.get_rank(group) if rank is None else rank
            self.ipc = IpcAllGather(n_local, world, r, group, self.x.device, dtype)
            self.y = torch.empty(1, n_local, dtype=dtype, device=device)
            self.rows = torch.empty(1, world * n_local, dtype=dtype, device=device)
        elif gather == "rccl":
            # At M = 1 the gathered [world, 1, n] IS the assembled [1, world * n] row in memory, and this rank's slice
            # of it can be the GEMV's output: the GEMV writes straight into place, the all-gather runs in place
            # (send buffer = receive buffer + rank * n), and nothing is copied -- one kernel per step at world 1
            # (round 3 had the GEMV + two copies).
            r = (dist.get_rank(group) if dist.is_available() and dist.is_initialized() else 0) if rank is None else rank
            self.y = self.gathered[r]
            self.rows = self.gathered.view(1, world * n_local)
        else:
            raise ValueError(f"ShardedDecode: unknown gather {gather!r}")

    def set_input(self, x: torch.Tensor):
        self.x.copy_(x.reshape(self.x.shape))

    def check(self):
        """Raise if the IPC gather of any step so far timed out (no-op for the RCCL gather, whose errors raise)."""
        if self.ipc is not None:
            self.ipc.check()

    def _barrier(self):
        if self.world > 1 and dist.is_available() and dist.is_initialized():
            dist.barrier(group=self.group)

    def step(self) -> torch.Tensor:
        """One eager decode step on the static buffers; returns `rows`."""
        self.local_fn(self.x, self.y)
        if self.ipc is not None:
            self.ipc(self.y, self.rows)
            if self.checked:
                self.ipc.check()
            return self.rows
        if _collective(self.world):
            if dist.get_backend(self.group) == "gloo":
                dist.all_gather(list(self.gathered.unbind(0)), self.y.clone(), group=self.group)
            else:
                dist.all_gather_into_tensor(self.gathered, self.y, group=self.group)   # in place
        return self.rows

    def capture(self, warmup: int = 2) -> bool:
        """Capture step() into a HIP graph (side-stream warm-up first, as torch.cuda.graph requires).  Returns False
        (and leaves eager mode) when the backend cannot be captured (gloo, or a collective capture refused)."""
        if not self.x.is_cuda or (self.ipc is None and _collective(self.world) and dist.get_backend(self.group) == "gloo"):
            return False
        # IPC: the warm-up steps wait on every peer's flags, so all ranks enter them together (a rank still loading or
        # capturing something else could otherwise exceed the bounded wait), and their outcome is checked before the
        # graph bakes the exchange in
        ipc = self.ipc is not None
        if ipc:
            self._barrier()
        s = torch.cuda.Stream(device=self.x.device)
        s.wait_stream(torch.cuda.current_stream(self.x.device))
        checked, self.checked = self.checked, False      # (no host sync inside the side stream / the capture)
        try:
            with torch.cuda.stream(s):
                for _ in range(warmup):
                    self.step()
            torch.cuda.current_stream(self.x.device).wait_stream(s)
            torch.cuda.synchronize(self.x.device)
            if ipc:
                self.ipc.check_all()      # every rank raises together, or none (a collective; also the barrier)
            g = torch.cuda.CUDAGraph()
            captured = True
            try:
                with torch.cuda.graph(g):
                    self.step()
            except Exception:  # noqa: BLE001 - capture refused: stay eager
                torch.cuda.synchronize(self.x.device)
                captured = False
        finally:
            self.checked = checked
        if ipc:
            self.ipc.check_all()          # reached on every rank, captured or not
        if not captured:
            return False
        self.graph = g
        return True

    def __call__(self, x: Optional[torch.Tensor] = None) -> torch.Tensor:
        if x is not None:
            self.set_input(x)
        if self.graph is not None:
            self.graph.replay()
            if self.checked:
                self.check()
            return self.rows
        return self.step()


class ColumnShardedLinear8bitLt(torch.nn.Module):
    """LLM.int8 counterpart: this rank holds rows [start, end) of CB/SCB; every rank quantises the
    replicated activations itself (int8_row_quant: no exchange), runs the fused igemmlt + dequant on its rows, and
    one RCCL all-gather assembles the fp16 output columns."""

    def __init__(self, CB: torch.Tensor, SCB: torch.Tensor, world: int, rank: int, group=None,
                 bias: Optional[torch.Tensor] = None):
        super().__init__()
        self.world, self.rank, self.group = world, rank, group
        self.out_features, self.in_features = CB.shape
        self.start, self.end = shard_range(self.out_features, world, rank)
        self.CB, self.SCB = shard_int8_rows(CB, SCB, world, rank)
        self.CB = self.CB.contiguous()
        self.bias = None if bias is None else bias[self.start:self.end].contiguous()

    @classmethod
    def from_linear(cls, layer, world: int, rank: int, group=None) -> "ColumnShardedLinear8bitLt":
        """Shard a quantised nn.Linear8bitLt (after .cuda(): CB/SCB on the weight, or in its state after a
        forward)."""
        CB = layer.weight.CB if layer.weight.CB is not None else layer.state.CB
        SCB = layer.weight.SCB if layer.weight.SCB is not None else layer.state.SCB
        bias = None if layer.bias is None else layer.bias.data.half()
        return cls(CB, SCB, world, rank, group, bias)

    def forward_local(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        x2 = x.reshape(-1, self.in_features)
        if x2.dtype != torch.float16:
            x2 = x2.half()
        CA, SCA = F.int8_row_quant(x2)
        return F.igemmlt_dequant(CA, self.CB, SCA, self.SCB, bias=self.bias, out=out)

    def forward(self, x: torch.Tensor, assemble: bool = True, chunks: int = 1) -> torch.Tensor:
        x2 = x.reshape(-1, self.in_features)
        if chunks > 1:
            mm = lambda xc, yc: self.forward_local(xc, yc)  # noqa: E731
            if not assemble:
                return sharded_forward_overlapped(x2, mm, self.world, self.group, chunks)
            rows = torch.empty((x2.shape[0], self.out_features), dtype=torch.float16, device=x2.device)
            return sharded_forward_overlapped(x2, mm, self.world, self.group, chunks, rows_out=rows)
        g = gather_columns(self.forward_local(x2), self.world, self.group)
        return gathered_to_rows(g) if assemble else g
