"""World-size-2 gloo test of the column-shard + all-gather logic (CPU, no GPU compute).

Each rank slices its rows out of a full 4-bit quantised weight with the product's
`shard_packed_rows`, computes its [M, N/2] output slice with the oracle (test-side compute),
and the product's `gather_columns` / `gathered_to_rows` assemble [M, N]; the result must equal
the unsharded oracle output bit-for-bit, and each slice must equal quantising the shard alone.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ret):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "bitsandbytes-sycl_amd")]
    from oracle import ref
    from python_src_quants.parallel import gather_columns, gathered_to_rows, shard_packed_rows, shard_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, K, M, bs = 96, 256, 5, 64
        rng = np.random.default_rng(0)
        W = (rng.standard_normal((N, K)) * 0.05).astype(np.float32)
        X = rng.standard_normal((M, K)).astype(np.float32)
        absmax, q = ref.quantize_blockwise(W.reshape(-1), bs, "nf4")
        start, end = shard_range(N, world, rank)
        p, a = shard_packed_rows(torch.from_numpy(q).reshape(-1, 1), torch.from_numpy(absmax), (N, K), bs, start, end)
        a_s, q_s = ref.quantize_blockwise(W[start:end].reshape(-1), bs, "nf4")
        assert np.array_equal(p.numpy().reshape(-1), q_s) and np.array_equal(a.numpy(), a_s)
        y_local = ref.gemm_4bit_dequant_ref(X, p.numpy(), a.numpy(), end - start, K, bs, ref.nf4_table(), "fp32")
        g = gather_columns(torch.from_numpy(y_local.astype(np.float32)), world)
        full = gathered_to_rows(g).numpy()
        exp = ref.gemm_4bit_dequant_ref(X, q, absmax, N, K, bs, ref.nf4_table(), "fp32").astype(np.float32)
        ret[rank] = bool(np.array_equal(full, exp))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_column_shard_allgather_gloo(world):
    port = _free_port()
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, port, ret), nprocs=world, join=True)
    assert dict(ret) == {r: True for r in range(world)}


def test_shard_range_errors():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "bitsandbytes-sycl_amd")]
    from python_src_quants.parallel import shard_range
    assert shard_range(4096, 8, 7) == (3584, 4096)
    with pytest.raises(ValueError):
        shard_range(100, 8, 0)


def _worker_overlap(rank, world, port, ret):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "bitsandbytes-sycl_amd")]
    from oracle import ref
    from python_src_quants.parallel import (chunked_to_rows, shard_packed_rows, shard_range,
                                            sharded_forward_overlapped)

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, K, M, bs = 64, 128, 12, 64
        rng = np.random.default_rng(1)
        W = (rng.standard_normal((N, K)) * 0.05).astype(np.float32)
        X = rng.standard_normal((M, K)).astype(np.float32)
        absmax, q = ref.quantize_blockwise(W.reshape(-1), bs, "nf4")
        start, end = shard_range(N, world, rank)
        p, a = shard_packed_rows(torch.from_numpy(q).reshape(-1, 1), torch.from_numpy(absmax), (N, K), bs, start, end)
        exp = ref.gemm_4bit_dequant_ref(X, q, absmax, N, K, bs, ref.nf4_table(), "fp32").astype(np.float32)

        def local_mm(xc, yc):   # test-side compute (the oracle) for this rank's rows
            y = ref.gemm_4bit_dequant_ref(xc.numpy(), p.numpy(), a.numpy(), end - start, K, bs, ref.nf4_table(), "fp32")
            return torch.from_numpy(y.astype(np.float32))
        ok = True
        for chunks in (1, 2, 3, 5):          # 5 does not divide M -> one chunk
            g = sharded_forward_overlapped(torch.from_numpy(X), local_mm, world, chunks=chunks)
            ok &= g.shape[0] == (chunks if M % chunks == 0 else 1)
            ok &= bool(np.array_equal(chunked_to_rows(g).numpy(), exp))
            full = torch.full((M, N), float("nan"))
            r = sharded_forward_overlapped(torch.from_numpy(X), local_mm, world, chunks=chunks, rows_out=full)
            ok &= r is full and bool(np.array_equal(full.numpy(), exp))
        ret[rank] = ok
    finally:
        dist.destroy_process_group()


def test_overlapped_chunked_allgather_gloo():
    """Row-chunked sharded forward with async all-gathers (the bench's multi-GPU step) assembles the
    unsharded result exactly for every chunk count."""
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker_overlap, args=(world, port, ret), nprocs=world, join=True)
    assert all(ret[r] for r in range(world))


def _worker_nested(rank, world, port, ret):
    """Each rank shards a NESTED quantised weight with the product's shard_quantized_4bit (no float weight), on CPU
    tensors: sliced second level when the shard starts on a 256-block boundary, re-compressed otherwise."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "bitsandbytes-sycl_amd")]
    from oracle import ref
    import python_src_quants.functional as F
    from python_src_quants.parallel import gather_columns, gathered_to_rows, shard_quantized_4bit

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ok = True
        bs = 64
        # (N, K): 512 x 64 -> 256 rows per rank = 256 blocks (aligned); 24 x 128 -> 12 rows = 24 blocks (not)
        for N, K, aligned in ((512, 64, True), (24, 128, False)):
            M = 3
            rng = np.random.default_rng(N)
            W = (rng.standard_normal((N, K)) * 0.05).astype(np.float32)
            X = rng.standard_normal((M, K)).astype(np.float32)
            absmax, q = ref.quantize_blockwise(W.reshape(-1), bs, "nf4")
            am = torch.from_numpy(absmax)
            offset = am.mean()
            qam, st2 = F.quantize_blockwise(am - offset, blocksize=256)       # the product's CPU path
            state = F.QuantState(absmax=qam, shape=torch.Size([N, K]), code=torch.from_numpy(ref.nf4_table()),
                                 blocksize=bs, quant_type="nf4", dtype=torch.float32, offset=offset, state2=st2)
            decoded = F._absmax_fp32(state).numpy()
            p, sst = shard_quantized_4bit(torch.from_numpy(q).reshape(-1, 1), state, world, rank)
            n = N // world
            ok &= tuple(sst.shape) == (n, K) and sst.nested
            ok &= bool(np.array_equal(p.numpy().reshape(-1), q[rank * n * K // 2:(rank + 1) * n * K // 2]))
            part = F._absmax_fp32(sst).numpy()
            full = decoded[rank * n * K // bs:(rank + 1) * n * K // bs]
            if aligned:
                ok &= bool(np.array_equal(part, full))
            else:
                ok &= bool(np.abs(part - full).max() <= 0.02 * np.abs(full).max())
            y_local = ref.gemm_4bit_dequant_ref(X, p.numpy(), part, n, K, bs, ref.nf4_table(), "fp32")
            g = gather_columns(torch.from_numpy(y_local.astype(np.float32)), world)
            got = gathered_to_rows(g).numpy()
            if aligned:
                exp = ref.gemm_4bit_dequant_ref(X, q, decoded, N, K, bs, ref.nf4_table(), "fp32").astype(np.float32)
                ok &= bool(np.array_equal(got, exp))
            else:
                exp = ref.gemm_4bit_dequant_ref(X, q, absmax, N, K, bs, ref.nf4_table(), "fp32")
                ok &= bool(np.abs(got - exp).max() <= 0.05 * np.abs(exp).max())
        ret[rank] = ok
    finally:
        dist.destroy_process_group()


def test_nested_shard_from_quantized_gloo():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker_nested, args=(world, port, ret), nprocs=world, join=True)
    assert all(ret[r] for r in range(world))


def _worker_int8(rank, world, port, ret):
    """LLM.int8 output-feature shard: CB/SCB rows via the product's shard_int8_rows; activations quantised on every
    rank (replicated); the gathered fp16 output equals the unsharded igemmlt + mm_dequant bit for bit."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "bitsandbytes-sycl_amd")]
    from oracle import ref
    from python_src_quants.parallel import gather_columns, gathered_to_rows, shard_int8_rows, shard_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(7)
        M, N, K = 9, 64, 96
        A = (rng.standard_normal((M, K)) * 2).astype(np.float16)
        Wt = (rng.standard_normal((N, K)) * 0.1).astype(np.float16)
        rsW, csW, _ = ref.colrow_absmax(Wt)
        CB, _ = ref.double_quant(Wt, rsW, csW)
        rsA, csA, _ = ref.colrow_absmax(A)
        CA, _ = ref.double_quant(A, rsA, csA)
        cb, scb = shard_int8_rows(torch.from_numpy(CB), torch.from_numpy(rsW), world, rank)
        s, e = shard_range(N, world, rank)
        y_local = ref.mm_dequant(ref.igemmlt(CA, cb.numpy()), rsA, scb.numpy())
        g = gather_columns(torch.from_numpy(y_local), world)
        exp = ref.mm_dequant(ref.igemmlt(CA, CB), rsA, rsW)
        ret[rank] = bool(np.array_equal(gathered_to_rows(g).numpy(), exp)) and cb.shape == (e - s, K)
    finally:
        dist.destroy_process_group()


def test_int8_row_shard_gloo():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker_int8, args=(world, port, ret), nprocs=world, join=True)
    assert all(ret[r] for r in range(world))


def _worker_decode(rank, world, port, ret):
    """ShardedDecode (the M = 1 step the multi-GPU bench captures in a HIP graph) on CPU tensors over gloo: each rank's
    GEMV is the oracle's gemv_4bit of its shard; the static-buffer step gathers and assembles the full decode row."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "bitsandbytes-sycl_amd")]
    from oracle import ref
    from python_src_quants.parallel import ShardedDecode

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, K, bs = 96, 128, 64
        rng = np.random.default_rng(5)
        W = (rng.standard_normal((N, K)) * 0.05).astype(np.float32)
        absmax, q = ref.quantize_blockwise(W.reshape(-1), bs, "nf4")
        n = N // world
        qs = q[rank * n * K // 2:(rank + 1) * n * K // 2]
        am = absmax[rank * n * K // bs:(rank + 1) * n * K // bs]

        def local(x, y):
            y.copy_(torch.from_numpy(ref.gemv_4bit(x.numpy().reshape(-1), qs, am, n, K, bs,
                                                   ref.nf4_table()).astype(np.float32)).view(1, n))
        dec = ShardedDecode(local, K, n, world, dtype=torch.float32, device="cpu")
        ok = dec.capture() is False                      # gloo / CPU: eager
        for seed in (1, 2):
            x = rng.standard_normal(K).astype(np.float32)
            got = dec(torch.from_numpy(x).view(1, K)).numpy().reshape(-1)
            exp = ref.gemv_4bit(x, q, absmax, N, K, bs, ref.nf4_table()).astype(np.float32)
            ok &= bool(np.array_equal(got, exp))
        ret[rank] = ok
    finally:
        dist.destroy_process_group()


def test_sharded_decode_step_gloo():
    """The M = 1 sharded forward on static buffers (ShardedDecode): per-rank GEMV + one all-gather assembles the
    unsharded decode output exactly, repeatedly on the same buffers."""
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker_decode, args=(world, port, ret), nprocs=world, join=True)
    assert all(ret[r] for r in range(world))


def test_ipc_allgather_host_rules():
    """Host side of the one-shot decode all-gather (no GPU needed): the exchange buffer is 512 B of flags
    (flags[2 parities][64 ranks] u32) + 2 parities x world slots of 16-B-padded shards, the shard width must be whole
    16-B pieces and the dtype 16-bit -- rejected before any device call."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "bitsandbytes-sycl_amd")]
    import python_src_quants.functional as F
    from python_src_quants.parallel import IpcAllGather
    for world, n in ((2, 1024), (8, 1376), (8, 8), (64, 128)):
        assert F.lib.cipc_allgather_buffer_bytes(world, n, 2) == 512 + 2 * world * ((2 * n + 15) // 16 * 16)
    assert F.lib.cipc_handle_size() == 64
    with pytest.raises(ValueError):
        IpcAllGather(1001, 2, 0)
    with pytest.raises(ValueError):
        IpcAllGather(1024, 2, 0, dtype=torch.float32)
