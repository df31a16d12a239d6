"""Lab (GPU): rocBLAS solution search for the library GEMM of the 4-bit prefill path (Y[M, N] = X[M, K] @ W[N, K]^T,
bf16 in/out, fp32 compute), through ctypes on the rocBLAS that torch already loaded (nothing in the product uses
rocBLAS).  Per shape: torch.matmul (hipBLASLt default), rocblas_gemm_ex with the standard algorithm, and every
solution rocblas_gemm_ex_get_solutions lists (one timed call each, the best five re-timed).
Usage: python tools/rocblas_solutions_probe.py [MxNxK ...]"""
import ctypes as ct
import sys
import time

import torch

SHAPES = [(4096, 11008, 4096), (4096, 4096, 11008), (2048, 4096, 11008)]
if len(sys.argv) > 1:
    SHAPES = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]]

OP_N, OP_T = 111, 112
BF16, F32 = 168, 151
ALGO_STD, ALGO_IDX = 0, 1


def t_us(fn, it=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / it


def main():
    torch.zeros(1, device="cuda")
    rb = ct.CDLL("librocblas.so.5")
    h = ct.c_void_p()
    assert rb.rocblas_create_handle(ct.byref(h)) == 0
    assert rb.rocblas_set_stream(h, ct.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    alpha, beta = ct.c_float(1.0), ct.c_float(0.0)
    for (m, n, k) in SHAPES:
        X = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
        W = torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.02
        Y = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)

        def args():
            return [h, OP_T, OP_N, n, m, k, ct.byref(alpha), ct.c_void_p(W.data_ptr()), BF16, k,
                    ct.c_void_p(X.data_ptr()), BF16, k, ct.byref(beta), ct.c_void_p(Y.data_ptr()), BF16, n,
                    ct.c_void_p(Y.data_ptr()), BF16, n, F32]

        def gemm(algo, idx):
            st = rb.rocblas_gemm_ex(*args(), algo, ct.c_int32(idx), ct.c_uint32(0))
            if st != 0:
                raise RuntimeError(f"rocblas_gemm_ex status {st}")
        size = ct.c_int32(0)
        st = rb.rocblas_gemm_ex_get_solutions(*args(), ALGO_IDX, ct.c_uint32(0), None, ct.byref(size))
        sols = (ct.c_int32 * max(1, size.value))()
        st = rb.rocblas_gemm_ex_get_solutions(*args(), ALGO_IDX, ct.c_uint32(0), sols, ct.byref(size))
        ref = torch.matmul(X, W.t())
        t_end = time.perf_counter() + 1.0
        while time.perf_counter() < t_end:
            torch.matmul(X, W.t(), out=Y)
            torch.cuda.synchronize()
        t_lt = t_us(lambda: torch.matmul(X, W.t(), out=Y))
        t_std = t_us(lambda: gemm(ALGO_STD, 0))
        cand = []
        t0 = time.perf_counter()
        for i in range(size.value):
            idx = sols[i]
            try:
                cand.append((t_us(lambda: gemm(ALGO_IDX, idx), it=2), idx))
            except RuntimeError:
                pass
        cand.sort()
        best = [(t_us(lambda: gemm(ALGO_IDX, idx), it=10), idx) for _, idx in cand[:5]]
        best.sort()
        gemm(ALGO_IDX, best[0][1])
        torch.cuda.synchronize()
        ok = (Y.float() - ref.float()).abs().max().item() <= 1e-2 * ref.float().abs().max().item()
        f = 2.0 * m * n * k
        print(f"{m}x{n}x{k}: hipBLASLt default {t_lt:7.1f} us ({f / t_lt / 1e6:5.0f} TF)  rocBLAS standard "
              f"{t_std:7.1f} us  best of {size.value} solutions {best[0][0]:7.1f} us ({f / best[0][0] / 1e6:5.0f} TF, "
              f"index {best[0][1]}; search {time.perf_counter() - t0:.1f} s; result ok {ok})", flush=True)
    rb.rocblas_destroy_handle(h)


if __name__ == "__main__":
    main()
