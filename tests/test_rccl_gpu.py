"""The multi-GPU code path's collectives on ONE GPU: a world-size-1 "nccl" (= RCCL) process group with the all-gathers
forced on (parallel.set_force_collective), so RCCL init, all_gather_into_tensor, its async chunk overlap
(sharded_forward_overlapped) and its HIP-graph capture (ShardedDecode.capture) run on hardware exactly as in the
8-GPU step.  Results are checked against the oracle: the NF4 shard forward within the bf16 GEMM
tolerance (|d| <= 2e-2 * rms + 2e-2 * |ref|), the decode row within the GEMV tolerance, the int8
shard forward bit-exact against ref.mm_dequant(ref.igemmlt(...)).  One process; the group is torn down at the end."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from oracle import ref

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def rccl(dev):
    import python_src_quants.parallel as P
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    P.set_force_collective(True)
    try:
        yield dev
    finally:
        P.set_force_collective(False)
        torch.cuda.synchronize(dev)
        dist.destroy_process_group()


def _tol_ok(got, exp):
    rms = np.sqrt(np.mean(exp ** 2))
    return bool(np.all(np.abs(got - exp) <= 2e-2 * rms + 2e-2 * np.abs(exp)))


def test_gather_columns_rccl(rccl):
    from python_src_quants.parallel import gather_columns
    assert dist.get_backend() == "nccl"
    y = torch.randn(37, 96, device=rccl, dtype=torch.bfloat16)
    out = torch.full((1, 37, 96), float("nan"), device=rccl, dtype=torch.bfloat16)
    g = gather_columns(y, 1, out=out)
    torch.cuda.synchronize(rccl)
    assert g is out and torch.equal(out[0], y)


@pytest.mark.parametrize("chunks", [1, 2, 4])
def test_sharded_forward_overlapped_rccl(rccl, chunks):
    """ColumnShardedLinear4bit.forward with async RCCL gathers per token-row chunk (the bench's N > 1 step) at world 1."""
    import python_src_quants.functional as F
    from python_src_quants.parallel import ColumnShardedLinear4bit
    N, K, M = 512, 1024, 256
    g = torch.Generator(device=rccl).manual_seed(11)
    W = (torch.randn(N, K, device=rccl, generator=g) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    lin = ColumnShardedLinear4bit.from_quantized(q, st, 1, 0)
    X = torch.randn(M, K, device=rccl, dtype=torch.bfloat16, generator=g)
    Y = lin.forward(X, assemble=True, chunks=chunks)
    torch.cuda.synchronize(rccl)
    assert Y.shape == (M, N)
    exp = ref.gemm_4bit_dequant_ref(X.float().cpu().numpy(), q.cpu().numpy(), F._absmax_fp32(st).cpu().numpy(), N, K,
                                    64, st.code.cpu().numpy(), "bf16")
    assert _tol_ok(Y.float().cpu().numpy(), exp)


def test_sharded_decode_graph_rccl(rccl):
    """ShardedDecode: GEMV + RCCL all_gather_into_tensor + row assembly captured in ONE HIP graph and replayed with
    new inputs; every replay matches the oracle GEMV of the same input."""
    import python_src_quants.functional as F
    from python_src_quants.parallel import ColumnShardedLinear4bit
    N, K = 1024, 4096
    g = torch.Generator(device=rccl).manual_seed(12)
    W = (torch.randn(N, K, device=rccl, generator=g) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    lin = ColumnShardedLinear4bit.from_quantized(q, st, 1, 0)
    dec = lin.decode_step()
    dec.set_input(torch.randn(1, K, device=rccl, dtype=torch.bfloat16, generator=g))
    assert dec.capture(), "RCCL all-gather was not captured into the HIP graph"
    qn, am, code = q.cpu().numpy(), F._absmax_fp32(st).cpu().numpy(), st.code.cpu().numpy()
    for _ in range(3):
        x = torch.randn(1, K, device=rccl, dtype=torch.bfloat16, generator=g)
        row = dec(x)
        torch.cuda.synchronize(rccl)
        exp = ref.gemv_4bit(x.float().cpu().numpy().reshape(-1), qn, am, N, K, 64, code)
        assert _tol_ok(row.float().cpu().numpy().reshape(-1), exp)


def test_int8_sharded_forward_rccl(rccl):
    """ColumnShardedLinear8bitLt with chunked RCCL gathers: bit-exact against the oracle's igemmlt + mm_dequant."""
    import python_src_quants.functional as F
    from python_src_quants.parallel import ColumnShardedLinear8bitLt
    M, N, K = 512, 256, 1024
    g = torch.Generator(device=rccl).manual_seed(13)
    A = (torch.randn(M, K, device=rccl, generator=g) * 2).half()
    Wt = (torch.randn(N, K, device=rccl, generator=g) * 0.05).half()
    CB, _, SCB, _, _ = F.double_quant(Wt)
    lin = ColumnShardedLinear8bitLt(CB, SCB, 1, 0)
    Y = lin.forward(A, assemble=True, chunks=2)
    CA, SCA = F.int8_row_quant(A)
    torch.cuda.synchronize(rccl)
    exp = ref.mm_dequant(ref.igemmlt(CA.cpu().numpy(), CB.cpu().numpy()), SCA.cpu().numpy(), SCB.cpu().numpy())
    assert np.array_equal(Y.cpu().numpy(), exp)
