"""Benchmark: NF4 matmul TFLOPS (+ INT8 igemmlt TOPS) @ M=4096, N=4096, K=11008 on 1..8 MI355X.

A "step" = one pass of the hot path over one batch of synthetic input, through functional.gemm_4bit as
MatMul4Bit.forward calls it (ref:python_src_quants/autograd/_functions.py:507):
    k_dequantize_4bit_stream (NF4 -> bf16 weight, nested statistics decoded in the same launch)
    -> the hand-written bf16 GEMM k_hgemm  Y_r = X @ W_r^T  (MFMA)
    -> RCCL all-gather of the bf16 output shards (when --gpus > 1).
W [4096, 11008] is column-sharded by output feature across ranks (rank r owns rows
r*N/g .. (r+1)*N/g of W, quantised NF4 bs=64 with nested statistics, the Linear4bit
default); X [4096, 11008] bf16 is replicated.  Total work is fixed -> "scaling": "strong".

Prints ONE JSON line on rank 0 (driver contract).  Extra fields: int8 igemmlt TOPS
(metric shape and config 3 = 4096^3), the decode GEMV (config 2) GB/s, the config-1
dequantize GB/s, the roofline of the dominant kernel and the CPU baseline.

Launch:  python bench.py [--gpus 1 --steps 20 --warmup 5]
         python bench.py --gpus N        (N > 1, no launcher: starts N rank processes itself, see launch_ranks)
         python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
from __future__ import annotations

import argparse
import ctypes as ct
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def _gpus_arg(argv) -> int:
    """--gpus N / --gpus=N from the command line (1 when absent); nothing else is parsed here."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    return ap.parse_known_args(argv)[0].gpus


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_launch_cmd(argv, port: int) -> list:
    """The command that runs this bench as `gpus` rank processes on this node (one per GPU, torch.distributed.run on
    127.0.0.1, the same arguments) -- what the driver's N > 1 launch line does."""
    n = _gpus_arg(argv)
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def world_mismatch(argv, env) -> str:
    """A message when the launcher's WORLD_SIZE and --gpus disagree (the bench would otherwise measure a world size
    other than the one it reports), else ''."""
    if "WORLD_SIZE" not in env:
        return ""
    world, gpus = int(env["WORLD_SIZE"]), _gpus_arg(argv)
    if world != gpus:
        return (f"bench.py: WORLD_SIZE={world} from the launcher but --gpus {gpus}: launch {gpus} ranks "
                f"(--nproc-per-node {gpus}) or pass --gpus {world}")
    return ""


def launch_ranks(argv) -> None:
    """--gpus N > 1 without a launcher (no WORLD_SIZE): start the N rank processes as ONE child (torch.distributed.run,
    so each rank gets RANK / LOCAL_RANK / WORLD_SIZE and its own GPU) and exit with its status -- before this process
    touches the GPU or imports torch, so nothing here has initialised HIP when the child starts.  Rank 0 of the child
    prints the JSON line.  A WORLD_SIZE that disagrees with --gpus exits non-zero (see world_mismatch)."""
    msg = world_mismatch(argv, os.environ)
    if msg:
        print(msg, file=sys.stderr, flush=True)
        sys.exit(2)
    if "WORLD_SIZE" in os.environ or _gpus_arg(argv) <= 1:
        return
    env = dict(os.environ)
    # The hosts of this pool support only dmabuf IPC; HSA_ENABLE_IPC_MODE_LEGACY=0 selects it (the images export it
    # already, here and on the GPU box, so the driver's own torchrun line runs with the same value).  Kept for a launch
    # from a stripped environment: without it RCCL / hipIpc handles fail with 'hipIpcGetMemHandle: invalid argument'.
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    rc = subprocess.call(rank_launch_cmd(argv, _free_port()), env=env)
    sys.exit(rc)


if __name__ == "__main__":
    launch_ranks(sys.argv[1:])

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import python_src_quants.functional as F  # noqa: E402
from python_src_quants.parallel import (ColumnShardedLinear8bitLt, shard_quantized_4bit,  # noqa: E402
                                        sharded_forward_overlapped)

M, N, K = 4096, 4096, 11008
BS = 64
PEAK_BF16_TFLOPS = 2500.0       # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_INT8_TOPS = 5000.0         # dense int8 MFMA (2x bf16)
PEAK_HBM_GBS = 8000.0           # HBM3E spec


def _events():
    return torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


# Per-stage events (dequantise / GEMM split, the roofline's kernel time) are recorded on every STAGE_EVERY-th timed
# step only: an event record between two kernels costs the stream ~3-4 us on this stack, so five per step cost
# ~18 us of a 250 us step (tools/step_overhead.py, profiles/lab/r02_step_overhead.txt).
STAGE_EVERY = 10
# gemm_4bit(..., prefetch=...): each dequantise + k_hgemm step dequantises the next weight inside its GEMM (--prefetch;
# default: the unpipelined pair, one dequantise launch before each GEMM -- measured faster so far)
PREFETCH = [False]


class StepClock:
    """Step boundaries of the timed region as HIP events on the launching stream, recorded only around the sampled
    steps (every `every`-th), so a sampled step i lasts ev[i] -> ev[i+1].
    An event record between two kernels costs the stream ~3-4 us (tools/step_overhead.py), so a record at every one of
    the K + 1 boundaries cost ~1 % of the metric step; the sampled form keeps the median without it (round 6)."""

    def __init__(self, steps, every=1):
        self.every = max(1, every) if steps >= 2 * every else 1     # (short runs: every step)
        # sampled steps: i % every == every // 2, i.e. not the steps that carry the stage events (i % every == 0);
        # the events are made (and first recorded: the HIP event is created then) up front, not inside the timed steps
        self.off = self.every // 2
        self.ev = {b: torch.cuda.Event(enable_timing=True) for b in range(steps + 1)
                   if self.every == 1 or (b - self.off) % self.every in (0, 1)}
        for e in self.ev.values():
            e.record()
        torch.cuda.synchronize()
        self.n = 0

    def mark(self):
        e = self.ev.get(self.n)
        if e is not None:
            e.record()
        self.n += 1

    def median_ms(self):
        import statistics
        return statistics.median(self.ev[b].elapsed_time(self.ev[b + 1]) for b in sorted(self.ev)
                                 if (b - self.off) % self.every == 0 and b + 1 in self.ev and b + 1 < self.n)


def _time_loop(fn, iters, warmup=3, prewarm_s=0.0):
    """Seconds per call of fn over `iters` back-to-back calls (one event pair around all of them).  prewarm_s: run fn
    untimed for that long first -- a leg that follows an idle or latency-bound one (graph-replayed decode) otherwise
    times its first milliseconds while the chip is still ramping its clock under the new load (round 3: the int8 leg
    read 163.7 us for a kernel that traces at 137-144 us)."""
    t_end = time.perf_counter() + prewarm_s
    while time.perf_counter() < t_end:
        for _ in range(8):
            fn()
        torch.cuda.synchronize()
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = _events()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3    # seconds per call


INT8_PREWARM_S = 0.3


def bench_int8(dev, m, n, k, iters=50):
    """Fused igemmlt + int32->fp16 dequant (cigemmlt_row_dequant_fp16) on row-major int8 operands,
    plus the full LLM.int8 forward (double_quant of the activations + the fused GEMM)."""
    g = torch.Generator(device=dev).manual_seed(3)
    A = (torch.randn(m, k, device=dev, generator=g) * 2).half()
    Wt = (torch.randn(n, k, device=dev, generator=g) * 0.05).half()
    CB, _, SCB, _, _ = F.double_quant(Wt)
    del Wt
    CA, _, SCA, _, _ = F.double_quant(A)
    out = torch.empty(m, n, dtype=torch.float16, device=dev)
    t_gemm = _time_loop(lambda: F.igemmlt_dequant(CA, CB, SCA, SCB, out=out), iters, prewarm_s=INT8_PREWARM_S)

    def fwd():
        ca, _, sca, _, _ = F.double_quant(A)
        F.igemmlt_dequant(ca, CB, sca, SCB, out=out)
    t_fwd = _time_loop(fwd, max(5, iters // 2))

    def fwd_inference():      # MatMul8bitLt without grad and outliers: one-pass row quantisation
        ca, sca = F.int8_row_quant(A)
        F.igemmlt_dequant(ca, CB, sca, SCB, out=out)
    t_inf = _time_loop(fwd_inference, max(5, iters // 2))
    ops = 2.0 * m * n * k
    # the reference ABI's own flow (ref:autograd/_functions.py:394-398): A -> col32, B cached as col_turing,
    # cigemmlt_turing_32 (int32 col32 out), then cdequant_mm_int32_fp16 -- three launches per forward
    CxB, SB = F.transform(CB, "col_turing")
    C32A, SA = F.transform(CA, "col32")
    out32, Sout = F.igemmlt(C32A, CxB, SA, SB)
    t_tr = _time_loop(lambda: F.transform(CA, "col32"), iters)
    t_ig = _time_loop(lambda: F.igemmlt(C32A, CxB, SA, SB, out=out32, Sout=Sout), iters)
    t_mm = _time_loop(lambda: F.mm_dequant(out32, Sout, SCA, SCB, out=out), iters)
    abi = {"igemmlt_turing_32_us": t_ig * 1e6, "igemmlt_turing_32_tops": ops / t_ig / 1e12,
           "transform_col32_us": t_tr * 1e6, "mm_dequant_us": t_mm * 1e6,
           "flow_us": (t_tr + t_ig + t_mm) * 1e6,
           "note": "F.transform(CA,'col32') + F.igemmlt(C32A, CxB col_turing) + F.mm_dequant, B transformed once"}
    return {"shape": [m, n, k], "tops": ops / t_gemm / 1e12, "us": t_gemm * 1e6,
            "frac_of_int8_peak": ops / t_gemm / 1e12 / PEAK_INT8_TOPS,
            "forward_with_double_quant_us": t_fwd * 1e6, "forward_inference_row_quant_us": t_inf * 1e6,
            "reference_abi_path": abi}


def auto_chunks(world, requested=0):
    """Token-row chunks of the sharded step (their all-gathers overlap the next chunk's GEMM).  Two chunks hide at most
    half the gather but run the rank's GEMM as two half-height products, which costs more compute the narrower the
    shard (tools/shard_parts_probe.py, profiles/lab/r04_shard_compute.txt: dequantise + GEMM per rank 156.6 vs 239.8 us
    at world 2, 105.6 vs 147.5 at 4, 66.7 vs 126.5 at 8 for one vs two chunks).  Chunking pays while half the gather
    exceeds that extra: with the per-peer xGMI bound of SURVEY §8(e) (~16.8 / 8.4 / 4.2 MB per link) the gather is
    ~220 / ~110 / ~55 us at 2 / 4 / 8 GPUs -- two chunks at 2 and 4, one at 8."""
    if world <= 1:
        return 1
    if requested >= 1:
        return requested if M % requested == 0 else 1
    return 1 if world >= 8 else 2


# ---------------------------------------------------------------------------------------------------------------------
# Self-validation of the N > 1 step: a broken all-gather must not print a TFLOP/s number.  After the
# timed region every rank checks the step's own outputs:
#   (a) its shard Y_r equals its column block of the assembled [M, N] output BIT FOR BIT (an all-gather is a copy);
#   (b) the assembled output is the same on every rank (a position-weighted checksum of its bits, MIN == MAX);
#   (c) rank 0 recomputes a sample of rows of the world-1 product on the FULL weight and compares (NF4: within the
#       GEMM tolerance -- the product is not row-split invariant; int8: bit for bit -- exact int32 and a
#       per-element epilogue).
# Results are combined over ranks (SUM / MIN / MAX all-reduces), so every rank reaches the same verdict; main() exits
# non-zero on any mismatch after rank 0 printed the line (outputs_verified false).

GEMM_RTOL = 2e-2        # the GEMM tolerance of the parity tests: |d| <= atol + rtol |ref|,
GEMM_ATOL_RMS = 2e-2    # atol = 2e-2 * rms(ref) for bf16


def _bits(t):
    """The raw bits of a tensor as integers of the same width (bitwise comparison: -0 != +0, NaN == NaN)."""
    t = t.contiguous()
    return t.view({1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[t.element_size()])


def _dist_on() -> bool:
    return dist.is_available() and dist.is_initialized()


def _reduce_int(v, op, dev):
    if not _dist_on():
        return int(v)
    t = torch.tensor([int(v)], device=dev, dtype=torch.int64)
    dist.all_reduce(t, op=op)
    return int(t.item())


def bits_checksum(a) -> int:
    """Position-weighted sum of the bits of `a` (int64, no overflow below ~2^37 16-bit elements): two tensors with the
    same checksum on every rank are, for this check's purpose, the same tensor."""
    b = _bits(a).reshape(-1)
    total, step = 0, 1 << 24
    for s in range(0, b.numel(), step):
        part = b[s:s + step].to(torch.int64)
        w = torch.arange(s, s + part.numel(), device=part.device, dtype=torch.int64) % 65521 + 1
        total += int((part * w).sum().item())
    return total


def sample_rows(m, count=64):
    """`count` token rows spread over [0, m), first and last included."""
    count = min(count, m)
    return sorted({round(i * (m - 1) / max(1, count - 1)) for i in range(count)})


def within_tolerance(got, ref, rtol=GEMM_RTOL, atol_rms=GEMM_ATOL_RMS) -> dict:
    """The GEMM tolerance of the parity tests, as a dict for the JSON line."""
    ref = ref.float()
    d = (got.float() - ref).abs()
    atol = atol_rms * float(ref.pow(2).mean().sqrt())
    bad = int((~(d <= atol + rtol * ref.abs())).sum().item())
    return {"ok": bad == 0, "violations": bad, "max_abs_err": float(d.max()), "atol": atol, "rtol": rtol}


def verify_sharded_output(y_local, assembled, world, rank, dev, sample_fn=None) -> dict:
    """Checks (a)-(c) above for one sharded step.  y_local [M, n]: this rank's output shard; assembled [M, world * n]:
    this rank's copy of the gathered output; sample_fn(assembled) -> dict with "ok" (run on rank 0 only).  Every rank
    takes part in the same collectives whatever its local result, and gets the same combined verdict."""
    n = y_local.shape[1]
    blk = assembled[:, rank * n:(rank + 1) * n]
    mism = int((_bits(blk) != _bits(y_local)).sum().item())
    ck = bits_checksum(assembled)
    sample, sample_ok = None, 1
    if rank == 0 and sample_fn is not None:
        try:
            sample = sample_fn(assembled)
        except Exception as ex:  # noqa: BLE001 - a failing check is a failed verification, not a hang of the others
            sample = {"ok": False, "error": repr(ex)}
        sample_ok = int(bool(sample.get("ok")))
    mism_all = _reduce_int(mism, dist.ReduceOp.SUM, dev)
    same = _reduce_int(ck, dist.ReduceOp.MIN, dev) == _reduce_int(ck, dist.ReduceOp.MAX, dev)
    sample_ok = _reduce_int(sample_ok, dist.ReduceOp.MIN, dev)
    res = {"ok": mism_all == 0 and same and sample_ok == 1, "shard_block_mismatches": mism_all,
           "assembled_identical_on_all_ranks": same, "world1_sample_ok": bool(sample_ok)}
    if sample is not None:
        res["world1_sample"] = sample
    return res


def nf4_world1_sample(X, q_full, st_full, rows):
    """sample_fn for the NF4 step: the sampled rows of the assembled output against (1) the world-1 product of the
    product path (gemm_4bit on the full weight) and (2) an fp32 product of the dequantised full weight (dequantize_4bit is
    bit-exact against the oracle), both within the GEMM tolerance."""
    idx = torch.tensor(rows, device=X.device)
    xs = X.index_select(0, idx).contiguous()
    y1 = F.gemm_4bit(xs, q_full, st_full)
    Wd = F.dequantize_4bit(q_full, st_full).float()
    ref = xs.float() @ Wd.t()
    del Wd

    def check(assembled):
        got = assembled.index_select(0, idx)
        a, b = within_tolerance(got, ref), within_tolerance(got, y1)
        return {"rows": len(rows), "ok": a["ok"] and b["ok"], "vs_fp32_of_dequantized_weight": a,
                "vs_world1_gemm_4bit": b}
    return check


def int8_world1_sample(A, CB_full, SCB_full, rows):
    """sample_fn for the int8 leg: the world-1 fused igemmlt + dequant of the sampled rows on the FULL CB; int32 is exact
    and the dequant is per element, so the assembled rows must equal it bit for bit."""
    idx = torch.tensor(rows, device=A.device)
    ca, sca = F.int8_row_quant(A.index_select(0, idx).contiguous())
    y1 = F.igemmlt_dequant(ca, CB_full, sca, SCB_full)

    def check(assembled):
        got = assembled.index_select(0, idx)
        mism = int((_bits(got) != _bits(y1)).sum().item())
        return {"rows": len(rows), "ok": mism == 0, "bitwise_mismatches_vs_world1": mism}
    return check


def time_allgather(y_chunk, out_chunk, chunks, world, dev, iters=20) -> dict:
    """The step's all-gather alone: `chunks` gathers of one [Mc, n] shard chunk per step (the step's own buffers and
    backend), barrier-bracketed, max over ranks.  Bytes: what every rank receives ((world - 1) shards) per step."""
    from python_src_quants.parallel import _gather_async
    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
    for _ in range(3):
        _gather_async(out_chunk, y_chunk).wait()
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        for _ in range(chunks):
            _gather_async(out_chunk, y_chunk).wait()
    sync()
    dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    per = t.item() / iters
    shard_bytes = y_chunk.numel() * y_chunk.element_size() * chunks
    recv = shard_bytes * (world - 1)
    return {"us_per_step": per * 1e6, "bytes_received_per_rank_per_step": recv,
            "bytes_assembled_per_rank_per_step": shard_bytes * world, "chunks": chunks,
            "recv_gbs_per_rank": recv / per / 1e9,
            "note": "the step's own all-gathers alone (own timing, not the overlapped step); max over ranks"}


def dist_info(dev) -> dict:
    """What the communicator and the devices report: backend, world size, and every rank's device (PCI id, name) --
    N distinct GPUs expected on the driver's multi-GPU node."""
    me = {"rank": dist.get_rank(), "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "pid": os.getpid()}
    if dev.type == "cuda":
        p = torch.cuda.get_device_properties(dev)
        me.update({"device": dev.index, "name": p.name,
                   "pci": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
                   "uuid": str(getattr(p, "uuid", ""))})
    ranks = [None] * dist.get_world_size()
    dist.all_gather_object(ranks, me)
    pcis = [r.get("pci") for r in ranks]
    return {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "ranks": ranks,
            "distinct_gpus": len(set(pcis)) if None not in pcis else 0}


def backend_label() -> str:
    """The process group's backend as the line names it ("RCCL" for torch's "nccl" on ROCm)."""
    if not (dist.is_available() and dist.is_initialized()):
        return "none"
    b = dist.get_backend()
    return "RCCL" if b == "nccl" else b


def verify_check_cpu(args, world, rank) -> int:
    """--verify-check: the N > 1 self-validation on CPU tensors over gloo (no GPU): the real sharded step helper
    (parallel.sharded_forward_overlapped) on an fp32 toy GEMM, then verify_sharded_output.  --corrupt MODE injects a
    fault on rank --corrupt-rank: "shard" (its own output changed after the gather: check a), "assembled" (its copy of
    another rank's block: check b), "values" (its shard computed from a perturbed weight, gathered consistently: only the
    world-1 sample, check c, sees it).  Prints rank 0's verdict as JSON; returns the exit status (3 = mismatch)."""
    from python_src_quants.parallel import sharded_forward_overlapped
    dist.init_process_group("gloo")
    dev = torch.device("cpu")
    m, n_out, k = 64, 32 * world, 128
    g = torch.Generator().manual_seed(5)
    X = torch.randn(m, k, generator=g)
    W = torch.randn(n_out, k, generator=g) * 0.05
    n = n_out // world
    Wr = W[rank * n:(rank + 1) * n].clone()
    if args.corrupt == "values" and rank == args.corrupt_rank:
        Wr[0, 0] += 1.0
    chunks = 2
    Y = torch.empty(m, n)
    gathered = torch.empty(chunks, world, m // chunks, n)
    full = torch.empty(m, n_out)
    sharded_forward_overlapped(X, lambda xc, yc: torch.matmul(xc, Wr.t(), out=yc), world, None, chunks,
                               out=gathered, y=Y, rows_out=full)
    if args.corrupt == "shard" and rank == args.corrupt_rank:
        Y[3, 1] += 1.0
    if args.corrupt == "assembled" and rank == args.corrupt_rank:
        other = (rank + 1) % world
        full[5, other * n] += 1.0
    rows = sample_rows(m, 16)
    ref = X[rows] @ W.t()
    res = verify_sharded_output(Y, full, world, rank, dev,
                                sample_fn=lambda a: within_tolerance(a[rows], ref))
    info = dist_info(dev)
    if rank == 0:
        print(json.dumps({"outputs_verified": res["ok"], "verification": res, "distributed": info}), flush=True)
    dist.destroy_process_group()
    return 0 if res["ok"] else 3


def bench_int8_sharded(dev, world, rank, steps, warmup, chunks, m=M, n=N, k=K):
    """The metric's INT8 half at 1/2/4/8 GPUs: Linear8bitLt's CB/SCB [n, k] sharded by output
    feature (ColumnShardedLinear8bitLt, rows of CB), the fp16 activations replicated and row-quantised on every
    rank (int8_row_quant, no exchange), the fused igemmlt + dequant on the rank's rows, one RCCL all-gather of the
    fp16 output (token-row chunks overlap the gather with the next chunk's GEMM).  Same barrier + max-over-ranks
    timing as the main step; TOPS = 2*m*n*k / step time (whole job)."""
    g = torch.Generator(device=dev).manual_seed(3)
    A = (torch.randn(m, k, device=dev, generator=g) * 2).half()
    Wt = (torch.randn(n, k, device=dev, generator=g) * 0.05).half()
    CB, _, SCB, _, _ = F.double_quant(Wt)
    del Wt
    lin = ColumnShardedLinear8bitLt(CB, SCB, world, rank)
    # rank 0 keeps the full CB / SCB for the world-1 sample check after the timed region (verify_sharded_output)
    check = int8_world1_sample(A, CB, SCB, sample_rows(m)) if world > 1 and rank == 0 else None
    del CB
    # (no per-step event chain here: an event record between two kernels costs the stream ~3-4 us, 2-3 % of this step;
    # the world-1 step writes into a preallocated output like a model's static buffer)
    out_local = torch.empty(m, lin.end - lin.start, dtype=torch.float16, device=dev) if world == 1 else None

    def step():
        if world > 1:
            lin.forward(A, assemble=True, chunks=chunks)
        else:
            lin.forward_local(A, out=out_local)
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    per = elapsed / steps
    ops = 2.0 * m * n * k
    res = {"shape": [m, n, k], "n_gpus": world, "tops": ops / per / 1e12, "ms_per_step": per * 1e3,
           "step": "int8_row_quant(X) + fused igemmlt+dequant on this rank's CB rows" +
                   (f" + {backend_label()} all_gather ({chunks} chunks) + [M, N] assembly" if world > 1 else ""),
           "frac_of_int8_peak": ops / per / 1e12 / PEAK_INT8_TOPS}
    if world > 1:
        # the step once more, outside the timed region, its outputs checked: this rank's rows alone (bit-exact whatever
        # the chunking: exact int32, per-element dequant) against its block of the assembled output
        assembled = lin.forward(A, assemble=True, chunks=chunks)
        local = lin.forward_local(A)
        torch.cuda.synchronize()
        res["verification"] = verify_sharded_output(local, assembled, world, rank, dev, sample_fn=check)
        res["outputs_verified"] = res["verification"]["ok"]
    return res


def bench_decode_sharded(dev, world, rank, steps, warmup, gather="rccl"):
    """Decode (M = 1) on `world` GPUs: the config-2 weight (Linear4bit NF4 11008 x 4096, nested statistics) sharded by
    output feature (ColumnShardedLinear4bit.from_quantized), one step = this rank's GEMV + ONE RCCL all-gather of the
    [1, 11008/world] bf16 shard outputs + the [1, 11008] row assembled (parallel.ShardedDecode, static buffers),
    captured in one HIP graph and replayed.  At M = 1 the all-gather moves KB and is latency-bound, so
    this reports latency: us per token for the layer, max over ranks, barrier-bracketed like the main step.  Ranks
    agree on the capture (all must succeed, else every rank replays the same step eagerly).  gather="ipc": the one-shot
    peer-memory all-gather (parallel.IpcAllGather) in place of RCCL; the result then carries the assembled row of a
    fixed input ("_row", for the caller's cross-check against the RCCL leg) and the polls that timed out."""
    from python_src_quants.parallel import ColumnShardedLinear4bit
    n_out, k_in = 11008, 4096
    g = torch.Generator(device=dev).manual_seed(2)
    W = (torch.randn(n_out, k_in, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=BS, quant_type="nf4", compress_statistics=True)
    del W
    lin = ColumnShardedLinear4bit.from_quantized(q, st, world, rank)
    lin.qweight = lin.qweight.clone()
    x_check = torch.randn(1, k_in, device=dev, dtype=torch.bfloat16, generator=g)
    ref_row = None
    if world > 1 and rank == 0:    # the world-1 row of x_check (fp32 product of the dequantised full weight)
        ref_row = x_check.float() @ F.dequantize_4bit(q, st).float().t()
    del q
    dec = lin.decode_step(gather=gather)
    dec.set_input(x_check)
    graph = dec.capture()
    if world > 1:
        ok = torch.tensor([1 if graph else 0], device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if ok.item() == 0:
            dec.graph, graph = None, False
    for _ in range(max(warmup, 3)):
        dec()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        dec()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    per = elapsed / steps
    n = n_out // world
    wbytes = n * k_in // 2 + n * k_in // BS + n * k_in // BS // 256 * 4 + 1024
    res = {"shape": [1, n_out, k_in], "n_gpus": world, "us_per_token": per * 1e6, "hip_graph": bool(graph),
           "weight_bytes_per_rank": wbytes, "rank_weight_gbs": wbytes / per / 1e9,
           "step": "gemv_4bit on this rank's rows" + (
               " + one-shot peer-memory all-gather (IpcAllGather, one kernel) into the [1, N] row" if gather == "ipc"
               else f" written into its slice of the [1, N] row + in-place {backend_label()} all_gather" if world > 1
               else " written straight into the [1, N] row (one kernel)"),
           "note": "host wall per replayed step (barrier-bracketed, max over ranks): the latency a decode token pays "
                   "for this one layer, including the graph launch"}
    dec.set_input(x_check)
    res["_row"] = dec().clone()
    torch.cuda.synchronize()
    if world > 1:
        # the assembled row against this rank's GEMV run on its own (same kernel and shape: bitwise), identical on every
        # rank, and (rank 0) against the world-1 row within the GEMM tolerance
        own = F.gemv_4bit(x_check, lin.qweight.t(), state=lin.quant_state)
        torch.cuda.synchronize()
        res["verification"] = verify_sharded_output(
            own, res["_row"], world, rank, dev,
            sample_fn=(lambda a: within_tolerance(a, ref_row)) if ref_row is not None else None)
        res["outputs_verified"] = res["verification"]["ok"]
    if dec.ipc is not None:
        res["ipc_timeouts"] = dec.ipc.timeouts()
        res["ipc_memory"] = dec.ipc.memory_kind
        dec.graph = None
        dec.ipc.close()
    # The same step for `layers` distinct layers (own weight copies and buffers) captured in ONE graph, as a model's
    # per-token graph holds all its layers: the per-layer latency without one graph launch per layer.  Every layer gets
    # the same input, so every layer's row must equal the single step's bit for bit.
    if graph:
        from python_src_quants.parallel import ShardedDecode
        layers = 8

        def make(qw):
            fn = lambda x, y: F.gemv_4bit(x, qw.t(), out=y, state=lin.quant_state)  # noqa: E731
            return ShardedDecode(fn, lin.in_features, lin.end - lin.start, world, None, torch.bfloat16, dev,
                                 gather=gather, rank=rank)
        decs = [make(lin.qweight.clone()) for _ in range(layers)]
        for d in decs:
            d.set_input(x_check)
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(2):
                for d in decs:
                    d.step()
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        gl, ok = torch.cuda.CUDAGraph(), 1
        try:
            with torch.cuda.graph(gl):
                for d in decs:
                    d.step()
        except Exception:  # noqa: BLE001 - capture refused: no multi-layer number
            ok = 0
        if world > 1:
            t = torch.tensor([ok], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            ok = int(t.item())
        if ok:
            for _ in range(max(warmup, 3)):
                gl.replay()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                gl.replay()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            if world > 1:
                t = torch.tensor([el], device=dev, dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                el = t.item()
            res["us_per_layer_in_graph"] = el / steps / layers * 1e6
            res["layers_per_graph"] = layers
            res["layers_match_single_step_bitwise"] = all(torch.equal(d.rows, res["_row"]) for d in decs)
        del gl
        for d in decs:
            if d.ipc is not None:
                res["ipc_timeouts"] = res.get("ipc_timeouts", 0) + d.ipc.timeouts()
                d.ipc.close()
    return res


def _time_graph(calls, iters):
    """Capture one pass over `calls` (distinct buffers each) into a HIP graph and time replays, so the
    number is the kernels' back-to-back time rather than the Python launch rate."""
    for c in calls:
        c()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for c in calls:
            c()
    t = _time_loop(g.replay, iters, warmup=2)
    return t / len(calls)


def bench_decode_gemv(dev, iters=30):
    """Config 2: Linear4bit NF4 decode M=1, K=4096, N=11008, bf16.  Both statistics formats: nested
    (compress_statistics=True, the Linear4bit default; decoded inside the GEMV kernel) and plain fp32.
    14 rotating weight copies (>256 MiB MALL) replayed from one HIP graph; GB/s over algorithmic bytes."""
    n_out, k_in = 11008, 4096
    copies = 14
    g = torch.Generator(device=dev).manual_seed(2)
    x = torch.randn(1, k_in, device=dev, dtype=torch.bfloat16, generator=g)
    out = torch.empty(1, n_out, device=dev, dtype=torch.bfloat16)
    res = {"shape": [1, n_out, k_in]}
    for nested in (True, False):
        ws = []
        for _ in range(copies):
            W = (torch.randn(n_out, k_in, device=dev, generator=g) * 0.02).to(torch.bfloat16)
            ws.append(F.quantize_4bit(W, blocksize=BS, quant_type="nf4", compress_statistics=nested))
            del W
        calls = [(lambda q=q, st=st: F.gemv_4bit(x, q.t(), out=out, state=st)) for q, st in ws]
        t = _time_graph(calls, iters)
        if nested:   # packed + 1-B codes + fp32 per 256 blocks + 1 KiB map + offset + x + out
            nbytes = n_out * k_in // 2 + n_out * k_in // BS + n_out * k_in // BS // 256 * 4 + 1024 + 4 + k_in * 2 + n_out * 2
        else:
            nbytes = n_out * k_in // 2 + n_out * k_in // BS * 4 + k_in * 2 + n_out * 2     # 25,392,640 B
        res["nested" if nested else "plain"] = {"us": t * 1e6, "gbs": nbytes / t / 1e9,
                                                "frac_of_hbm": nbytes / t / 1e9 / PEAK_HBM_GBS, "bytes": nbytes}
        del ws
    res["note"] = "14 rotating weight copies (~355 MB) defeat the 256 MB MALL; HIP-graph replay (kernel time)"
    return res


def bench_few_token_gemm(dev, iters=30, tokens=(2, 4, 8, 16, 32, 64)):
    """Batched decode / short prefill on the config-2 weight (11008 x 4096 NF4, nested statistics, the
    Linear4bit default): gemm_4bit with 2..32 activation rows runs the whole-K few-token kernel (gemm4bit_fewtok.hip,
    one launch), 33..64 the split-K weight-streaming kernel (gemm4bit_skinny.hip, + its ordered reduce).  14 rotating weight copies, HIP-graph replay;
    GB/s over the algorithmic bytes (packed weights + nested stats + activations + output)."""
    n_out, k_in, copies = 11008, 4096, 14
    g = torch.Generator(device=dev).manual_seed(3)
    ws = []
    for _ in range(copies):
        W = (torch.randn(n_out, k_in, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        ws.append(F.quantize_4bit(W, blocksize=BS, quant_type="nf4", compress_statistics=True))
        del W
    res = {"shape": [None, n_out, k_in],
           "path": "2..32 rows: k_gemm_4bit_fewtok (whole K per workgroup, LDS-DMA weight ring, 16x16x32 MFMA, one "
                   "launch); 33..64 rows: k_gemm_4bit_t64 (192 weight rows x 64 tokens per workgroup, split-K, "
                   "+ k_skinny_reduce)"}
    for m in tokens:
        x = torch.randn(m, k_in, device=dev, dtype=torch.bfloat16, generator=g)
        out = torch.empty(m, n_out, device=dev, dtype=torch.bfloat16)
        calls = [(lambda q=q, st=st: F.gemm_4bit(x, q, st, out=out)) for q, st in ws]
        t = _time_graph(calls, iters)
        nbytes = (n_out * k_in // 2 + n_out * k_in // BS + n_out * k_in // BS // 256 * 4 + 1024 + 4
                  + m * k_in * 2 + m * n_out * 2)
        res[f"tokens_{m}"] = {"us": t * 1e6, "gbs": nbytes / t / 1e9, "frac_of_hbm": nbytes / t / 1e9 / PEAK_HBM_GBS,
                              "tflops": 2.0 * m * n_out * k_in / t / 1e12}
    res["note"] = "14 rotating weight copies (~355 MB) defeat the 256 MB MALL; HIP-graph replay (kernel time)"
    return res


def bench_dequant_config1(dev, iters=30):
    """Config 1 on the GPU: dequantize_blockwise NF4 of a 4096x4096 weight, bs=64 -> bf16 (HBM-bound)."""
    g = torch.Generator(device=dev).manual_seed(0)
    copies = 30       # 30 x 9.4 MB of packed input > 256 MB MALL
    qs = []
    for _ in range(copies):
        W = torch.randn(4096, 4096, device=dev, generator=g)
        qs.append(F.quantize_4bit(W, blocksize=BS, quant_type="nf4"))
    outs = [torch.empty(4096, 4096, device=dev, dtype=torch.bfloat16) for _ in range(2)]

    def call(q, st, o):
        F.pre_call(dev)      # binds the library to the current (capturing) stream
        F.lib.cdequantize_blockwise_bf16_nf4(None, F.get_ptr(q), F.get_ptr(st.absmax), F.get_ptr(o), ct.c_int(BS),
                                             ct.c_int(4096 * 4096))
    calls = [(lambda q=q, st=st, o=outs[i % 2]: call(q, st, o)) for i, (q, st) in enumerate(qs)]
    t = _time_graph(calls, iters)
    nbytes = 42_991_616
    return {"us": t * 1e6, "gbs": nbytes / t / 1e9, "frac_of_hbm": nbytes / t / 1e9 / PEAK_HBM_GBS, "bytes": nbytes}


def bench_optimizer_8bit(dev, n=1 << 27, iters=10):
    """Adam with 8-bit blockwise states (c<T>adam_8bit_blockwise_grad), HBM-bound.
    Algorithmic bytes per element: g + p read, p write (sizeof T each), two state bytes read + written,
    plus 2 x 4 B of absmax per 2048-element block read + written."""
    res = {"n": n}
    q1 = F.create_dynamic_map(signed=True).to(dev)
    q2 = F.create_dynamic_map(signed=False).to(dev)
    for dt, name in ((torch.float32, "fp32"), (torch.bfloat16, "bf16")):
        g = torch.Generator(device=dev).manual_seed(9)
        p = (torch.randn(n, device=dev, generator=g) * 0.1).to(dt)
        grad = (torch.randn(n, device=dev, generator=g) * 0.01).to(dt)
        s1 = torch.zeros(n, dtype=torch.uint8, device=dev)
        s2 = torch.zeros(n, dtype=torch.uint8, device=dev)
        blocks = (n + 2047) // 2048
        a1 = torch.zeros(blocks, device=dev)
        a2 = torch.zeros(blocks, device=dev)
        step = [0]

        def call():
            step[0] += 1
            F.optimizer_update_8bit_blockwise("adam", grad, p, s1, s2, 0.9, 0.999, 1e-8, step[0], 1e-3, q1, q2, a1, a2)
        t = _time_loop(call, iters)
        esz = p.element_size()
        nbytes = n * (3 * esz + 4) + blocks * 16
        res[name] = {"us": t * 1e6, "gbs": nbytes / t / 1e9, "frac_of_hbm": nbytes / t / 1e9 / PEAK_HBM_GBS,
                     "bytes": nbytes}
        del p, grad, s1, s2
    # the fp32-state Adam (c<T>adam32bit_grad) on the same parameters: g + p read, p write, two fp32 states
    # read + written -- pure streaming, the HBM reference point for the 8-bit kernels above
    g = torch.Generator(device=dev).manual_seed(9)
    p = (torch.randn(n, device=dev, generator=g) * 0.1)
    grad = (torch.randn(n, device=dev, generator=g) * 0.01)
    s1 = torch.zeros(n, device=dev)
    s2 = torch.zeros(n, device=dev)
    step = [0]

    def call32():
        step[0] += 1
        F.optimizer_update_32bit("adam", grad, p, s1, 0.9, 1e-8, step[0], 1e-3, state2=s2, beta2=0.999)
    t = _time_loop(call32, iters)
    nbytes = n * 28
    res["fp32_states_fp32"] = {"us": t * 1e6, "gbs": nbytes / t / 1e9, "frac_of_hbm": nbytes / t / 1e9 / PEAK_HBM_GBS,
                               "bytes": nbytes}
    del p, grad, s1, s2
    return res


def bench_nf4_fused_kernel(dev, m=M, n=N, k=K, iters=20):
    """The hand-written fused NF4 GEMM (cgemm_4bit_inference_code_ws_bf16: dequantise in LDS + bf16
    MFMA) at the metric shape, forced (functional.gemm_4bit routes this size to dequantise + hipBLASLt)."""
    g = torch.Generator(device=dev).manual_seed(4)
    X = torch.randn(m, k, device=dev, dtype=torch.bfloat16, generator=g)
    W = (torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=BS, quant_type="nf4", compress_statistics=True)
    del W
    Y = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    am = F._absmax_fp32(st)
    t = _time_loop(lambda: F.gemm_4bit(X, q, st, out=Y, absmax=am, _route="fused"), iters)
    flops = 2.0 * m * n * k
    return {"shape": [m, n, k], "kernel": "k_gemm_4bit_256<bf16>", "us": t * 1e6, "tflops": flops / t / 1e12,
            "frac_of_bf16_peak": flops / t / 1e12 / PEAK_BF16_TFLOPS}


def bench_llama2_7b_prefill(dev, batch=32, seq=2048, iters=3):
    """Config 4: the seven Linear4bit NF4 projections of one Llama-2-7B decoder layer (q, k, v, o: 4096 ->
    4096; gate, up: 4096 -> 11008; down: 11008 -> 4096; bs=64, nested statistics) at batch 32 x seq 2048
    = 65,536 tokens, bf16, through functional.gemm_4bit (all 32 layers have these shapes; per-layer time)."""
    tokens = batch * seq
    hid, inter = 4096, 11008
    g = torch.Generator(device=dev).manual_seed(6)
    shapes = [(hid, hid)] * 4 + [(inter, hid)] * 2 + [(hid, inter)]
    ws = []
    for n_out, k_in in shapes:
        W = (torch.randn(n_out, k_in, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        ws.append(F.quantize_4bit(W, blocksize=BS, quant_type="nf4", compress_statistics=True))
        del W
    X = torch.randn(tokens, hid, device=dev, dtype=torch.bfloat16, generator=g)
    Xi = torch.randn(tokens, inter, device=dev, dtype=torch.bfloat16, generator=g)
    outs = {n_out: torch.empty(tokens, n_out, device=dev, dtype=torch.bfloat16) for n_out in (hid, inter)}

    def layer():
        # each projection's GEMM dequantises the next one's weight (the last: the next layer's first, same shapes)
        for i, ((n_out, k_in), (q, st)) in enumerate(zip(shapes, ws)):
            F.gemm_4bit(X if k_in == hid else Xi, q, st, out=outs[n_out],
                        prefetch=ws[(i + 1) % len(ws)] if PREFETCH[0] else None)
    t = _time_loop(layer, iters)
    flops = sum(2.0 * tokens * n_out * k_in for n_out, k_in in shapes)
    res = {"tokens": tokens, "layer_ms": t * 1e3, "tflops": flops / t / 1e12, "model_32_layers_ms": 32 * t * 1e3,
           "path": gemm_kernel_name(tokens, hid)}
    del X, Xi, outs, ws
    torch.cuda.empty_cache()
    return res


def bench_llama2_70b_shard(dev, ranks=8, prefill_tokens=4096, layer_copies=8, iters=3):
    """Config 5 on one GPU: the rank-local work of one Llama-2-70B decoder layer column-sharded 8 ways (the seven
    Linear4bit NF4 projections, nested statistics; hidden 8192, GQA k/v 1024, MLP 28672; each rank holds N/8 output
    columns: q/o 1024 x 8192, k/v 128 x 8192, gate/up 3584 x 8192, down 1024 x 28672), at a 4096-token prefill and
    at 1-token decode, through functional.gemm_4bit / gemv_4bit as Linear4bit calls them.  The bf16 all-gather of
    the shards (parallel.py) is not in these numbers: the multi-GPU bench times it.  Decode: `layer_copies` distinct
    layers (> the 256 MB MALL) replayed from one HIP graph, GB/s over the packed weights + statistics read."""
    hid, kv, inter = 8192, 1024, 28672
    shapes = [(hid // ranks, hid), (kv // ranks, hid), (kv // ranks, hid), (hid // ranks, hid),
              (inter // ranks, hid), (inter // ranks, hid), (hid // ranks, inter)]
    g = torch.Generator(device=dev).manual_seed(8)
    layers = []
    for _ in range(layer_copies):
        ws = []
        for n_out, k_in in shapes:
            W = (torch.randn(n_out, k_in, device=dev, generator=g) * 0.02).to(torch.bfloat16)
            ws.append(F.quantize_4bit(W, blocksize=BS, quant_type="nf4", compress_statistics=True))
            del W
        layers.append(ws)
    res = {"rank_shapes": [[n, k] for n, k in shapes], "ranks": ranks}
    # prefill: one layer, 4096 tokens
    X = torch.randn(prefill_tokens, hid, device=dev, dtype=torch.bfloat16, generator=g)
    Xi = torch.randn(prefill_tokens, inter, device=dev, dtype=torch.bfloat16, generator=g)
    outs = {n: torch.empty(prefill_tokens, n, device=dev, dtype=torch.bfloat16) for n, _ in shapes}

    def layer():
        ws = layers[0]
        for i, ((n_out, k_in), (q, st)) in enumerate(zip(shapes, ws)):
            F.gemm_4bit(X if k_in == hid else Xi, q, st, out=outs[n_out],
                        prefetch=ws[(i + 1) % len(ws)] if PREFETCH[0] else None)
    t = _time_loop(layer, iters)
    flops = sum(2.0 * prefill_tokens * n * k for n, k in shapes)
    res["prefill"] = {"tokens": prefill_tokens, "layer_ms": t * 1e3, "tflops": flops / t / 1e12,
                      "model_80_layers_ms": 80 * t * 1e3}
    del X, Xi, outs
    # decode: one token through every projection of `layer_copies` layers
    x, xi = (torch.randn(1, k, device=dev, dtype=torch.bfloat16, generator=g) for k in (hid, inter))
    dec_out = {n: torch.empty(1, n, device=dev, dtype=torch.bfloat16) for n, _ in shapes}
    calls = [(lambda q=q, st=st, n=n, k=k: F.gemv_4bit(x if k == hid else xi, q.t(), out=dec_out[n], state=st))
             for ws in layers for (n, k), (q, st) in zip(shapes, ws)]
    t_call = _time_graph(calls, 10)
    t_layer = t_call * len(shapes)
    wbytes = sum(n * k // 2 + n * k // BS + n * k // BS // 256 * 4 + 1024 for n, k in shapes)
    res["decode"] = {"layer_us": t_layer * 1e6, "weight_bytes_per_layer": wbytes, "gbs": wbytes / t_layer / 1e9,
                     "frac_of_hbm": wbytes / t_layer / 1e9 / PEAK_HBM_GBS, "model_80_layers_ms": 80 * t_layer * 1e3}
    # the same layers with the projections that share an input fused (parallel.fuse_quantized_4bit): q/k/v one
    # 1280 x 8192 weight, gate/up one 7168 x 8192 -- four launches per layer instead of seven
    from python_src_quants.parallel import fuse_quantized_4bit
    fused = []
    for ws in layers:
        qkv = fuse_quantized_4bit([ws[0], ws[1], ws[2]])[:2]
        gu = fuse_quantized_4bit([ws[4], ws[5]])[:2]
        fused.append([qkv, ws[3], gu, ws[6]])
    fshapes = [(shapes[0][0] + shapes[1][0] + shapes[2][0], hid), shapes[3], (2 * shapes[4][0], hid), shapes[6]]
    fout = {i: torch.empty(1, n, device=dev, dtype=torch.bfloat16) for i, (n, _) in enumerate(fshapes)}
    fcalls = [(lambda q=q, st=st, i=i, k=k: F.gemv_4bit(x if k == hid else xi, q.t(), out=fout[i], state=st))
              for ws in fused for i, ((n, k), (q, st)) in enumerate(zip(fshapes, ws))]
    tf = _time_graph(fcalls, 10) * len(fshapes)
    fbytes = sum(n * k // 2 + n * k // BS + n * k // BS // 256 * 4 + 1024 for n, k in fshapes)
    res["decode_fused"] = {"layer_us": tf * 1e6, "launches_per_layer": len(fshapes), "weight_bytes_per_layer": fbytes,
                           "gbs": fbytes / tf / 1e9, "frac_of_hbm": fbytes / tf / 1e9 / PEAK_HBM_GBS,
                           "model_80_layers_ms": 80 * tf * 1e3,
                           "fused": "q/k/v -> 1280 x 8192, gate/up -> 7168 x 8192 (parallel.fuse_quantized_4bit)"}
    del fused, fcalls
    res["note"] = ("rank-local compute only (no all-gather); decode over 8 distinct layers (~430 MB) from one HIP "
                   "graph; prefill path per shape from the measured route")
    del layers, calls
    torch.cuda.empty_cache()
    return res


def host_cpu_info():
    """The GPU box's host CPU as the bench sees it: model name (/proc/cpuinfo), logical CPUs of the machine and
    the CPUs this process may run on (the box gives a job a share of a larger machine)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    return {"model": model, "nproc_machine": os.cpu_count(), "cpus_usable": usable,
            "torch_threads": torch.get_num_threads()}


def cpu_baseline(rows=M, budget_s=12.0, max_reps=40):
    """Reference CPU path as ported (oracle/cpu_ops_port.cpp, the restated cpu_ops.cpp dequantize_cpu,
    single-threaded as written) + torch CPU F.linear (the CPU path has no GEMM), on a
    bounded sample: per repetition the full W [4096, 11008] is dequantised and multiplied with `rows`
    activation rows (all M = 4096 by default: the whole metric product, no extrapolation); repetitions run until
    ~budget_s of CPU work, the median rep is reported.  Threads: torch's, i.e. the job's CPU share on the box (the pool
    sets OMP_NUM_THREADS to the per-GPU share, 16; the machine's other cores belong to other jobs' GPUs, so taking them
    would measure a neighbour's slowdown, not this baseline).  Beside it,
    config 1 itself (NF4 4096 x 4096, bs 64, one index byte per element) through the port and through the
    product's host entry point cdequantize_blockwise_cpu_fp32 (csrc/cpu_ops.cpp, multi-threaded)."""
    import numpy as np
    import statistics
    sys.path.insert(0, ROOT)
    from oracle.maps import nf4_padded_256
    lib = ct.CDLL(os.path.join(ROOT, "oracle", "_build", "libcpu_ops_port.so"))
    rng = np.random.default_rng(0)
    n_el = N * K
    idx = rng.integers(0, 16, n_el, dtype=np.uint8)            # unpacked NF4 indices, 1 B/elem (Q17)
    absmax = rng.uniform(0.01, 0.1, n_el // BS).astype(np.float32)
    code = nf4_padded_256()
    W = np.empty(n_el, np.float32)
    Wt = torch.from_numpy(W).view(N, K)
    X = torch.randn(rows, K)
    threads = torch.get_num_threads()
    torch.nn.functional.linear(X[:8], Wt)
    vp = lambda a: a.ctypes.data_as(ct.c_void_p)   # noqa: E731
    deq, mm = [], []
    start = time.perf_counter()
    while len(deq) < max_reps and (time.perf_counter() - start) < budget_s:
        t0 = time.perf_counter()
        lib.port_dequantize_cpu(vp(code), vp(idx), vp(absmax), vp(W), ct.c_longlong(BS), ct.c_longlong(n_el))
        t1 = time.perf_counter()
        torch.nn.functional.linear(X, Wt)
        t2 = time.perf_counter()
        deq.append(t1 - t0)
        mm.append(t2 - t1)
    t_deq, t_mm = statistics.median(deq), statistics.median(mm)
    flops = 2.0 * rows * N * K
    value = flops / (t_deq + t_mm) / 1e12

    # config 1 (4096 x 4096 NF4, bs 64): 16 MiB of index bytes + 1 MiB absmax -> 64 MiB fp32
    n1 = 4096 * 4096
    i1, a1, o1 = idx[:n1], absmax[:n1 // BS], W[:n1]
    c1_bytes = n1 + n1 // BS * 4 + n1 * 4
    t_port, t_prod = [], []
    # the product CPU path on the job's CPU share (torch's thread count), not every core of the machine
    prod_threads = int(F.lib.cset_cpu_threads(threads))
    for _ in range(5):
        t0 = time.perf_counter()
        lib.port_dequantize_cpu(vp(code), vp(i1), vp(a1), vp(o1), ct.c_longlong(BS), ct.c_longlong(n1))
        t1 = time.perf_counter()
        F.lib.cdequantize_blockwise_cpu_fp32(vp(code), vp(i1), vp(a1), vp(o1), ct.c_longlong(BS), ct.c_longlong(n1))
        t2 = time.perf_counter()
        t_port.append(t1 - t0)
        t_prod.append(t2 - t1)
    F.lib.cset_cpu_threads(0)
    tp, tq = statistics.median(t_port), statistics.median(t_prod)
    return {"value": value, "unit": "TFLOP/s", "cores": threads, "kind": "port",
            "sample": f"{len(deq)} reps of: dequantize_cpu (1 thread, as ref:sycl/cpu_ops.cpp:7-14) of W[{N},{K}] "
                      f"NF4 bs=64 unpacked ({t_deq:.3f}s, {n_el * 9 / t_deq / 1e9:.2f} GB/s) + torch CPU fp32 "
                      f"F.linear on {rows} of the {M} rows ({t_mm:.3f}s, {threads} torch threads = the job's CPU "
                      f"share, OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS')}); median rep",
            "cores_per_leg": {"dequantize_cpu": 1, "torch_linear": threads},
            "host": host_cpu_info(),
            "dequant_cpu_gbs": n_el * 9 / t_deq / 1e9,
            "config1_cpu": {"shape": [4096, 4096], "bytes": c1_bytes,
                            "port_1_thread": {"ms": tp * 1e3, "gbs": c1_bytes / tp / 1e9},
                            "product_cpu_path": {"ms": tq * 1e3, "gbs": c1_bytes / tq / 1e9, "threads": prod_threads,
                                                 "entry": "cdequantize_blockwise_cpu_fp32 (csrc/cpu_ops.cpp)"},
                            "note": "median of 5; same inputs; outputs bit-identical (tests/test_cpu_path.py)"}}


def gemm_kernel_name(m, n, k=K, route=None):
    """Which kernel carries gemm_4bit's flops for m tokens x n features: the route (measured when `route` is given,
    else functional.gemm_4bit_static_route) -- "hgemm": the hand-written k_hgemm after the dequantise kernel;
    "library" / "library_tn": the library GEMM after the dequantise kernel (torch's hipBLASLt pick / the
    rocBLAS-searched one); "fused": gemm4bit.hip's 256x256 tile kernel when the features are >= 256 and the grid (with
    split-K) has >= 128 workgroups, else the 128x128 one."""
    route = route or F.gemm_4bit_static_route(m, n, k)
    if route == "hgemm":
        if PREFETCH[0]:
            return ("k_hgemm<bf16> (hand-written, hgemm.hip) with the next call's NF4 dequantise inside it "
                    "(prefetch, HgSide)")
        return "k_hgemm<bf16> (hand-written, hgemm.hip) after k_dequantize_4bit_stream<bf16,NF4>"
    if route == "library_tn":
        return ("library bf16 GEMM (Cijk_*, rocBLAS solution searched per shape, cgemm_tn_bf16) after "
                "k_dequantize_4bit_stream<bf16,NF4>")
    if route == "library":
        return "library bf16 GEMM (Cijk_* hipBLASLt, via torch.matmul) after k_dequantize_4bit_stream<bf16,NF4>"
    ks = max(1, F.lib.cgemm_4bit_workspace_bytes(ct.c_int32(n), ct.c_int32(m), ct.c_int32(k)) // (4 * m * n))
    tiles256 = ((m + 255) // 256) * ((n + 255) // 256)
    tiles128 = ((m + 127) // 128) * ((n + 127) // 128)
    if n >= 256 and (tiles256 * ks >= 128 or 2 * tiles256 * ks >= tiles128):
        return "k_gemm_4bit_256<bf16>" + (f" split-K x{ks} + k_splitk_reduce" if ks > 1 else "")
    return "k_gemm_4bit<bf16>"


def dequant_route(kname):
    """True when the kernel carrying the flops runs after the dequantise kernel (statistics decoded there)."""
    return kname.startswith("library") or kname.startswith("k_hgemm")


def measure_peaks(dev, reps=5):
    """Measured ceilings on this box (spec AND measured peak), from the library's probe kernels
    (csrc/probe.hip): the dense bf16 and int8 MFMA rate on random register operands at one wave per SIMD (the GEMMs'
    own shapes and occupancy), and the HBM streaming read rate over 2 GiB (> the 256 MB MALL).  Median of `reps`
    timed launches after a ~0.3 s clock ramp."""
    import statistics
    blocks = 256         # one workgroup per CU: 4 waves (one per SIMD) or 8 (two per SIMD)
    sink = torch.empty(blocks * 512, device=dev)
    res = {}
    for kind, name, per in ((0, "bf16_mfma_tflops", 16 * 16 * 32 * 2), (1, "int8_mfma_tops", 16 * 16 * 64 * 2)):
        best = {}
        for waves in (4, 8):
            k = kind + (2 if waves == 8 else 0)
            iters = 40000
            F.pre_call(dev)
            t_end = time.perf_counter() + 0.3
            while time.perf_counter() < t_end:
                F.lib.cprobe_mfma(k, blocks, iters, 7, F.get_ptr(sink))
                torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                s, e = _events()
                s.record()
                F.lib.cprobe_mfma(k, blocks, iters, 7, F.get_ptr(sink))
                e.record()
                e.synchronize()
                ts.append(s.elapsed_time(e) * 1e-3)
            best[waves] = blocks * waves * 8 * iters * per / statistics.median(ts) / 1e12
        res[name] = max(best.values())
        res[name + "_by_waves_per_cu"] = {str(w): round(v, 1) for w, v in best.items()}
    buf = torch.empty(1 << 31, dtype=torch.uint8, device=dev)
    hsink = torch.empty(4096, dtype=torch.int32, device=dev)
    ts = []
    for i in range(reps + 2):
        s, e = _events()
        s.record()
        F.lib.cprobe_hbm_read(F.get_ptr(buf), ct.c_longlong(buf.numel()), 4096, F.get_ptr(hsink))
        e.record()
        e.synchronize()
        if i >= 2:
            ts.append(s.elapsed_time(e) * 1e-3)
    res["hbm_read_gbs"] = buf.numel() / statistics.median(ts) / 1e9
    del buf
    torch.cuda.empty_cache()
    res["how"] = ("csrc/probe.hip: MFMA 16x16x32 bf16 / 16x16x64 i8 back to back on random register operands, one or two "
                  "waves per SIMD (the faster is the peak), 8 AGPR accumulators per wave; HBM: 16-B non-temporal loads, "
                  "8 in flight per lane, 2 GiB buffer")
    return res


def load_pmc_traffic():
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(p):
        try:
            with open(p) as f:
                return json.load(f)
        except Exception:  # noqa: BLE001
            return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)   # >= 100 launches after 10 warm-up
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-extras", action="store_true", help="skip int8/decode/config-1/cpu legs")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-int8", action="store_true", help="skip the sharded int8 leg")
    ap.add_argument("--no-decode", action="store_true", help="skip the sharded decode (M = 1) leg")
    ap.add_argument("--no-ipc", action="store_true", help="N > 1: skip the one-shot peer-memory decode all-gather leg")
    ap.add_argument("--prefetch", action="store_true",
                    help="dequantise each step's weight inside the previous step's GEMM (gemm_4bit prefetch=)")
    ap.add_argument("--prewarm-ms", type=float, default=400.0, help="untimed clock-ramp period before warmup")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, the product path); gloo only to rehearse N>1 ranks on one GPU")
    ap.add_argument("--chunks", type=int, default=0,
                    help="N>1: token-row chunks whose all-gathers overlap the next chunk's GEMM (0 = auto: 2 at 2 and "
                         "4 GPUs, 1 at 8 -- see auto_chunks)")
    ap.add_argument("--verify-check", action="store_true",
                    help="N>1 output self-validation on CPU tensors over gloo (no GPU); exits 3 on a mismatch")
    ap.add_argument("--corrupt", default="none", choices=("none", "shard", "assembled", "values"),
                    help="--verify-check: the fault to inject (see verify_check_cpu)")
    ap.add_argument("--corrupt-rank", type=int, default=1)
    ap.add_argument("--launch-check", action="store_true",
                    help="print the rank layout (every rank over gloo, no GPU work) and exit: checks the N-rank launch")
    args = ap.parse_args()
    PREFETCH[0] = args.prefetch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:       # (launch_ranks has already started the ranks / refused a mismatch; imported callers)
        raise SystemExit(world_mismatch(sys.argv[1:], os.environ) or
                         f"bench.py: world size {world} but --gpus {args.gpus}")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.verify_check:
        if world < 2:
            raise SystemExit("bench.py --verify-check needs --gpus N >= 2")
        sys.exit(verify_check_cpu(args, world, rank))
    if args.launch_check:
        # the rank layout only (no GPU): every rank joins a gloo group and rank 0 prints who took part
        if world > 1:
            dist.init_process_group("gloo")
        ranks = [None] * world
        if world > 1:
            dist.all_gather_object(ranks, {"rank": rank, "local_rank": local_rank, "pid": os.getpid()})
        else:
            ranks = [{"rank": 0, "local_rank": local_rank, "pid": os.getpid()}]
        if rank == 0:
            print(json.dumps({"n_gpus": world, "gpus_arg": args.gpus, "ranks": ranks}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    dev = torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
    assert N % world == 0
    shard = N // world

    # ---- synthetic data (same global problem for every world size)
    gx = torch.Generator(device=dev).manual_seed(1)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=gx)
    # the full weight, quantised once (nested statistics, the Linear4bit default) and sliced per rank by the
    # product's shard_quantized_4bit -- what a rank does with a pre-quantised checkpoint (no float weight)
    gw = torch.Generator(device=dev).manual_seed(1000)
    W = (torch.randn(N, K, device=dev, generator=gw) * 0.02).to(torch.bfloat16)
    q_full, st_full = F.quantize_4bit(W, blocksize=BS, quant_type="nf4", compress_statistics=True)
    del W
    q, st = shard_quantized_4bit(q_full, st_full, world, rank)
    # rank 0: the world-1 sample check after the timed region (verify_sharded_output) needs the full weight
    nf4_check = nf4_world1_sample(X, q_full, st_full, sample_rows(M)) if rank == 0 else None
    if world > 1:
        q = q.clone()
        del q_full
    Y = torch.empty(M, shard, device=dev, dtype=torch.bfloat16)
    chunks = auto_chunks(world, args.chunks)
    Mc = M // chunks
    gathered = torch.empty(chunks, world, Mc, shard, device=dev, dtype=torch.bfloat16) if world > 1 else None
    # N > 1: the step ends with the layer's [M, N] output assembled (chunk by chunk, as each gather lands)
    full_out = torch.empty(M, world * shard, device=dev, dtype=torch.bfloat16) if world > 1 else None
    kev = []

    library = dequant_route(gemm_kernel_name(Mc, shard))

    clock = StepClock(args.steps, STAGE_EVERY)
    F.reserve_stage_events(3 * (args.steps // STAGE_EVERY + 1))   # the sampled steps' stage events, made up front

    def step(record=False):
        # fused kernel: nested stats -> fp32 absmax once per step, shared by the chunks; library path:
        # gemm_4bit decodes them inside its dequantise launch
        absmax = None if library else F._absmax_fp32(st)
        ev = []

        first = [True]
        calls = [0]

        def mm(xc, yc):   # chunks after the first reuse this step's dequantised shard (library path)
            # the step's last GEMM dequantises the next step's weight inside it (prefetch; the layer's next weight in a
            # model -- here the same shard again, so every step still dequantises it once)
            calls[0] += 1
            pf = (q, st) if PREFETCH[0] and calls[0] == chunks else None
            r = F.gemm_4bit(xc, q, st, out=yc, absmax=absmax, events=ev if record else None,
                            reuse_weight=not first[0], prefetch=pf)
            first[0] = False
            return r
        if world > 1:
            # chunk c's RCCL all-gather (own stream) overlaps chunk c+1's GEMM; all waited at the end
            sharded_forward_overlapped(X, mm, world, None, chunks, out=gathered, y=Y, rows_out=full_out)
        else:
            mm(X, Y)
        if record:
            kev.append(ev)

    # clock ramp: MI355X takes ~0.1-0.3 s of sustained MFMA load to reach its steady clock; run the
    # step untimed for --prewarm-ms before the W counted warmup steps (the timed region is unchanged)
    # (GEMM only: a time-based loop must not contain a collective, ranks could disagree on its count)
    # first call of the shape (workspaces; under BNB_ROUTE_TUNING its route measurement): done before the clock-ramp
    # period starts, so the ramp is not spent on it
    F.gemm_4bit(X[:Mc], q, st, out=Y[:Mc], absmax=None if library else F._absmax_fp32(st))
    torch.cuda.synchronize()
    t_end = time.perf_counter() + args.prewarm_ms / 1e3
    while time.perf_counter() < t_end:
        am = None if library else F._absmax_fp32(st)
        for c in range(chunks):
            F.gemm_4bit(X[c * Mc:(c + 1) * Mc], q, st, out=Y[c * Mc:(c + 1) * Mc], absmax=am)
        torch.cuda.synchronize()
    # the route gemm_4bit takes for this shape (the static rule, or a measured one under BNB_ROUTE_TUNING)
    kname = gemm_kernel_name(Mc, shard, route=F.gemm_4bit_measured_route(X[:Mc], st))
    library = dequant_route(kname)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    clock.mark()
    for i in range(args.steps):
        step(record=(i % STAGE_EVERY == 0))
        clock.mark()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    ms_per_step = elapsed / args.steps * 1e3
    total_flops = 2.0 * M * N * K
    value = total_flops / (elapsed / args.steps) / 1e12
    # mean duration per chunk of the stage that carries the flops (the fused kernel incl. any split-K
    # reduce, or the library GEMM) and of the dequantise stage that precedes the library GEMM
    def stage_mean(name):
        d = [s.elapsed_time(e) for ev in kev for nm, s, e in ev if nm == name]
        return sum(d) / len(d) * 1e-3 if d else None
    kern_s = stage_mean("gemm")
    deq_s = stage_mean("dequantize")
    shard_flops = 2.0 * Mc * shard * K
    achieved = shard_flops / kern_s / 1e12

    median_step_ms = clock.median_ms()

    # N > 1: the step's own outputs checked (the last timed step's Y and assembled [M, N]), the communicator and the
    # devices recorded, the all-gather timed alone -- all outside the timed region
    verification, dinfo, allgather = None, None, None
    torch.cuda.synchronize()
    verification = verify_sharded_output(Y, full_out if world > 1 else Y, world, rank, dev, sample_fn=nf4_check)
    if world > 1:
        dinfo = dist_info(dev)
        allgather = time_allgather(Y[:Mc], gathered[0], chunks, world, dev)
        allgather["backend"] = backend_label()

    extras = {}
    if not args.no_int8:     # every rank: it contains collectives when world > 1
        extras["int8_igemmlt_sharded"] = bench_int8_sharded(dev, world, rank, args.steps, args.warmup, chunks)
    if not args.no_decode:   # every rank: the sharded decode step (GEMV + all-gather) as one HIP graph
        extras["decode_sharded_config2"] = bench_decode_sharded(dev, world, rank, args.steps, args.warmup)
        row_rccl = extras["decode_sharded_config2"].pop("_row")
        if world > 1 and not args.no_ipc:
            # the same step on the one-shot peer-memory all-gather; every rank takes part (exchange setup is collective)
            try:
                r_ipc = bench_decode_sharded(dev, world, rank, args.steps, args.warmup, gather="ipc")
                same = torch.tensor([1 if torch.equal(r_ipc.pop("_row"), row_rccl) else 0], device=dev)
                dist.all_reduce(same, op=dist.ReduceOp.MIN)
                r_ipc["matches_rccl_row_bitwise"] = bool(same.item())
                t = torch.tensor([r_ipc.get("ipc_timeouts", 0)], device=dev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                r_ipc["ipc_timeouts"] = int(t.item())
                if not r_ipc["matches_rccl_row_bitwise"] or r_ipc["ipc_timeouts"]:
                    r_ipc["valid"] = False
                extras["decode_sharded_config2_ipc"] = r_ipc
            except Exception as ex:  # noqa: BLE001
                extras["decode_sharded_config2_ipc"] = {"error": repr(ex)}
    if rank == 0 and world == 1 and not args.no_extras:
        extras["int8_igemmlt_metric_shape"] = bench_int8(dev, M, N, K)
        extras["int8_igemmlt_config3"] = bench_int8(dev, 4096, 4096, 4096)
        extras["decode_gemv_config2"] = bench_decode_gemv(dev)
        extras["few_token_gemm_config2_weight"] = bench_few_token_gemm(dev)
        extras["dequant_nf4_config1_gpu"] = bench_dequant_config1(dev)
        extras["optimizer_adam8bit_blockwise"] = bench_optimizer_8bit(dev)
        extras["nf4_fused_kernel_metric_shape"] = bench_nf4_fused_kernel(dev)
        extras["llama2_7b_prefill_config4"] = bench_llama2_7b_prefill(dev)
        extras["llama2_70b_rank_shard_config5"] = bench_llama2_70b_shard(dev)
    peaks = None
    if rank == 0 and not args.no_extras:
        try:
            peaks = measure_peaks(dev)
        except Exception as ex:  # noqa: BLE001
            peaks = {"error": str(ex)}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and not args.no_extras:
        try:
            cpu = cpu_baseline()
        except Exception as ex:  # noqa: BLE001
            cpu = {"value": None, "unit": "TFLOP/s", "cores": None, "kind": "port", "sample": f"failed: {ex}"}

    # every rank holds the same combined verdicts (verify_sharded_output all-reduces them)
    legs = {"nf4_step": verification}
    if world > 1:
        for key in ("int8_igemmlt_sharded", "decode_sharded_config2"):
            if key in extras:
                legs[key] = extras[key].get("verification")
    bad_legs = [k for k, v in legs.items() if not (v and v.get("ok"))]
    if rank == 0 and peaks and "int8_mfma_tops" in peaks:
        for key in ("int8_igemmlt_sharded", "int8_igemmlt_metric_shape", "int8_igemmlt_config3"):
            if key in extras and "tops" in extras[key]:
                extras[key]["frac_of_int8_peak_measured"] = extras[key]["tops"] / peaks["int8_mfma_tops"]
    if rank == 0:
        pmc = load_pmc_traffic()
        traffic = None
        pmc_extra = {}
        if pmc and pmc.get("kernel") == kname and pmc.get("shape") == [Mc, shard, K]:
            traffic = pmc.get("hbm_bytes_per_launch")
            pmc_extra = {k: pmc[k] for k in ("mfma_busy_per_simd", "effective_clock_ghz") if k in pmc}
        line = {
            "metric": "NF4 matmul TFLOPS + INT8 igemmlt TOPS @ 4096x4096x11008, 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "TFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "median_step_ms_rank0": round(median_step_ms, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (seeded randn; W ~ N(0,0.02) -> NF4 bs=64 nested stats; X ~ N(0,1) bf16)",
            "config": {"workload": "NF4 Linear4bit GEMM M=4096 N=4096 K=11008 (functional.gemm_4bit on its static "
                                   f"route for {Mc} x {shard} x {K}: {kname}"
                                   + ("; the dequantise of each step's weight run inside the previous step's k_hgemm "
                                      "(--prefetch)" if PREFETCH[0] else ", every step dequantising its weight") +
                                   ")" + (" + bf16 all-gather of output-column shards" if world > 1 else ""),
                       "M": M, "N": N, "K": K, "blocksize": BS, "quant_type": "nf4", "compress_statistics": True,
                       "parallelism": (f"column-shard x{world} + {backend_label()} all_gather, {chunks} token-row chunks "
                                       "(chunk c's all-gather overlaps chunk c+1's GEMM; the step ends with the [M, N] "
                                       "output assembled)") if world > 1 else "single GPU"},
            "roofline": {"bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
                         "peak_measured": round(peaks["bf16_mfma_tflops"], 1) if peaks and "bf16_mfma_tflops" in peaks
                         else None,
                         "frac_measured": round(achieved / peaks["bf16_mfma_tflops"], 4)
                         if peaks and "bf16_mfma_tflops" in peaks else None,
                         "kernel": kname, "kernel_us": round(kern_s * 1e6, 2),
                         "flops_per_launch": shard_flops,
                         "dequantize_us": round(deq_s * 1e6, 2) if deq_s else None,
                         # the step's dequantise runs inside the previous step's k_hgemm (kernel_us includes it)
                         "dequantize_inside_gemm": bool(PREFETCH[0] and kname.startswith("k_hgemm")), **pmc_extra},
            "measured_peaks": peaks,
            "cpu_baseline": cpu,
        }
        line["verification"] = verification
        if world > 1:
            line["distributed"] = dinfo
            line["allgather"] = allgather
        line["outputs_verified"] = not bad_legs
        if bad_legs:
            line["verification_failed"] = bad_legs
        line.update(extras)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if bad_legs:
        print(f"bench.py: output verification FAILED on {bad_legs} (rank {rank})", file=sys.stderr, flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
