"""The one-shot decode all-gather over peer memory (parallel.IpcAllGather, csrc/ipc.hip callgather_ipc_16) with TWO
processes on the box's one GPU: each process allocates its exchange buffer, the hipIpc handles travel over a gloo
group, each opens the other's buffer, and every step pushes a rank-specific [1, n] slice; the assembled [1, 2n] row
must equal the two slices side by side (rank j's columns at j * n) bit for bit, eagerly and replayed from a HIP graph
with new inputs, with no poll timing out.  Then a ShardedDecode(gather="ipc") step of a real NF4 shard pair against
the oracle GEMV.  (Two ranks on one device exercise the handles, the flags, the epochs / parities and the graph
capture; xGMI itself needs the driver's multi-GPU run.)  A second test pins the fail-stop behaviour: a step whose peer
never pushes gives up after the bounded wait and writes a NaN row (not the stale slots), check() raises, and every
later step of that exchange stays NaN without waiting again."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


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
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    try:
        import python_src_quants.functional as F
        from oracle import ref
        from python_src_quants.parallel import ColumnShardedLinear4bit, IpcAllGather
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        n = 1376                                   # 11008 / 8: one 8-way shard of the config-2 decode row
        ag = IpcAllGather(n, world, rank, device=dev)
        res["kind"] = ag.memory_kind
        y = torch.empty(1, n, device=dev, dtype=torch.bfloat16)
        rows = torch.empty(1, world * n, device=dev, dtype=torch.bfloat16)
        ok = True
        for step in range(6):                      # eager: epochs 1..6, both parities
            y.copy_(torch.full((1, n), float(10 * step + rank), device=dev) +
                    torch.arange(n, device=dev).view(1, n) * 1e-2)
            dist.barrier()
            ag(y, rows)
            torch.cuda.synchronize()
            exp = torch.cat([torch.full((1, n), float(10 * step + r), device=dev) +
                             torch.arange(n, device=dev).view(1, n) * 1e-2 for r in range(world)], 1).to(torch.bfloat16)
            ok &= torch.equal(rows, exp)
        # graph capture of the step (the way ShardedDecode replays it), replayed with new inputs
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            ag(y, rows)
        for step in range(6, 10):
            y.copy_(torch.full((1, n), float(step * 3 + rank), device=dev))
            torch.cuda.synchronize()
            dist.barrier()
            g.replay()
            torch.cuda.synchronize()
            exp = torch.cat([torch.full((1, n), float(step * 3 + r), device=dev) for r in range(world)], 1)
            ok &= torch.equal(rows, exp.to(torch.bfloat16))
        res["raw"] = bool(ok)
        res["timeouts"] = ag.timeouts()
        ag.close()
        # a ShardedDecode step on the one-shot gather: the full NF4 decode row against the oracle GEMV
        N, K = 2048, 1024
        gw = torch.Generator(device=dev).manual_seed(31)
        W = (torch.randn(N, K, device=dev, generator=gw) * 0.02).to(torch.bfloat16)
        q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
        lin = ColumnShardedLinear4bit.from_quantized(q, st, world, rank)
        dec = lin.decode_step(gather="ipc")
        x = torch.randn(1, K, device=dev, dtype=torch.bfloat16, generator=gw)
        dist.barrier()
        row = dec(x)
        torch.cuda.synchronize()
        e = ref.gemv_4bit(x.float().cpu().numpy().reshape(-1), q.cpu().numpy(), F._absmax_fp32(st).cpu().numpy(), N, K,
                          64, st.code.cpu().numpy())
        got = row.float().cpu().numpy().reshape(-1)
        rms = np.sqrt(np.mean(e ** 2))
        res["decode"] = bool(np.all(np.abs(got - e) <= 2e-2 * rms + 2e-2 * np.abs(e)))
        res["decode_timeouts"] = dec.ipc.timeouts()
        dec.ipc.close()
    except Exception as ex:  # noqa: BLE001
        res["error"] = repr(ex)
    finally:
        ret[rank] = res
        dist.destroy_process_group()


def _timeout_worker(rank, world, port, ret):
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "bitsandbytes-sycl_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    try:
        from python_src_quants.parallel import IpcAllGather
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        n = 64
        ag = IpcAllGather(n, world, rank, device=dev)
        res["kind"] = ag.memory_kind
        y = torch.full((1, n), float(rank + 1), device=dev, dtype=torch.bfloat16)
        rows = torch.zeros(1, world * n, device=dev, dtype=torch.bfloat16)
        dist.barrier()
        ag(y, rows)                                # a healthy step first
        torch.cuda.synchronize()
        res["healthy"] = bool(torch.equal(rows.float().view(world, n),
                                          torch.arange(1, world + 1, device=dev).float().view(world, 1).expand(world, n)))
        dist.barrier()
        if rank == 0:                              # rank 1 never pushes this step: bounded wait, then poison
            t0 = time.perf_counter()
            ag(y, rows)
            torch.cuda.synchronize()
            res["wait_s"] = time.perf_counter() - t0
            res["nan_row"] = bool(torch.isnan(rows.float()).all())
            res["timeouts"] = ag.timeouts()
            try:
                ag.check()
                res["raised"] = False
            except RuntimeError:
                res["raised"] = True
            rows.zero_()
            t0 = time.perf_counter()
            ag(y, rows)                            # latched: NaN at once, no second wait
            torch.cuda.synchronize()
            res["latched_s"] = time.perf_counter() - t0
            res["latched_nan"] = bool(torch.isnan(rows.float()).all())
            res["timeouts_after"] = ag.timeouts()
        dist.barrier()
        try:                                       # the agreed check: rank 1 timed out nowhere, yet raises too
            ag.check_all()
            res["all_raised"] = False
        except RuntimeError:
            res["all_raised"] = True
        dist.barrier()
        ag.close()
    except Exception as ex:  # noqa: BLE001
        res["error"] = repr(ex)
    finally:
        ret[rank] = res
        dist.destroy_process_group()


def test_ipc_allgather_timeout_poisons_row():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_timeout_worker, args=(world, port, ret), nprocs=world, join=True)
    got = dict(ret)
    for r in range(world):
        assert "error" not in got[r], got[r]
        assert got[r]["kind"] == "uncached" and got[r]["healthy"], got[r]
    r0 = got[0]
    assert r0["nan_row"] and r0["timeouts"] >= 1 and r0["raised"], r0
    assert r0["latched_nan"] and r0["timeouts_after"] == r0["timeouts"], r0
    assert r0["latched_s"] < 0.25 * r0["wait_s"], r0
    assert all(got[r]["all_raised"] for r in range(world)), got     # check_all: every rank raises together


def test_ipc_allgather_two_processes_one_gpu():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, port, ret), nprocs=world, join=True)
    got = dict(ret)
    for r in range(world):
        assert "error" not in got[r], got[r]
        assert got[r]["kind"] == "uncached", got[r]
        assert got[r]["raw"] and got[r]["timeouts"] == 0, got[r]
        assert got[r]["decode"] and got[r]["decode_timeouts"] == 0, got[r]
