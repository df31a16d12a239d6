"""Lab (GPU): rocBLAS solution search for the int8 GEMM of igemmlt (C[M, N] int32 = A[M, K] int8 . B[N, K]^T int8),
through ctypes on the rocBLAS that torch already loaded.  Per shape: torch._int_mm (hipBLASLt), rocblas_gemm_ex with
the standard algorithm, and every solution rocblas_gemm_ex_get_solutions lists (one warm + one timed call each, the
best five re-timed); exactness against torch._int_mm.  Compare with k_igemm_256 (bench.py int8 legs).
Usage: python tools/rocblas_int8_probe.py [MxNxK ...]"""
import ctypes as ct
import sys
import time

import torch

SHAPES = [(4096, 4096, 11008), (4096, 4096, 4096)]
if len(sys.argv) > 1:
    SHAPES = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]]

OP_N, OP_T = 111, 112
I8, I32 = 160, 162
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
    alpha, beta = ct.c_int32(1), ct.c_int32(0)
    for (m, n, k) in SHAPES:
        X = torch.randint(-127, 128, (m, k), device="cuda", dtype=torch.int8)
        W = torch.randint(-127, 128, (n, k), device="cuda", dtype=torch.int8)
        Y = torch.empty(m, n, device="cuda", dtype=torch.int32)

        def args():
            return [h, OP_T, OP_N, n, m, k, ct.byref(alpha), ct.c_void_p(W.data_ptr()), I8, k,
                    ct.c_void_p(X.data_ptr()), I8, k, ct.byref(beta), ct.c_void_p(Y.data_ptr()), I32, n,
                    ct.c_void_p(Y.data_ptr()), I32, n, I32]

        def gemm(algo, idx):
            st = rb.rocblas_gemm_ex(*args(), algo, ct.c_int32(idx), ct.c_uint32(0))
            if st != 0:
                raise RuntimeError(f"rocblas_gemm_ex status {st}")
        size = ct.c_int32(0)
        st = rb.rocblas_gemm_ex_get_solutions(*args(), ALGO_IDX, ct.c_uint32(0), None, ct.byref(size))
        sols = (ct.c_int32 * max(1, size.value))()
        st = rb.rocblas_gemm_ex_get_solutions(*args(), ALGO_IDX, ct.c_uint32(0), sols, ct.byref(size))
        ref = torch._int_mm(X, W.t())
        t_end = time.perf_counter() + 1.0
        while time.perf_counter() < t_end:
            torch._int_mm(X, W.t())
            torch.cuda.synchronize()
        t_lt = t_us(lambda: torch._int_mm(X, W.t()))
        t_std = t_us(lambda: gemm(ALGO_STD, 0))
        cand = []
        t0 = time.perf_counter()
        for i in range(size.value):
            idx = sols[i]
            try:
                gemm(ALGO_IDX, idx)
                cand.append((t_us(lambda: gemm(ALGO_IDX, idx), it=2), idx))
            except RuntimeError:
                pass
        cand.sort()
        best = [(t_us(lambda: gemm(ALGO_IDX, idx), it=10), idx) for _, idx in cand[:5]]
        best.sort()
        if not best:
            gemm(ALGO_STD, 0)
            torch.cuda.synchronize()
            print(f"{m}x{n}x{k}: _int_mm {t_lt:7.1f} us  rocBLAS standard {t_std:7.1f} us (exact "
                  f"{torch.equal(Y, ref)}); {size.value} solutions listed, none ran", flush=True)
            continue
        gemm(ALGO_IDX, best[0][1])
        torch.cuda.synchronize()
        ok = torch.equal(Y, ref)
        f = 2.0 * m * n * k
        print(f"{m}x{n}x{k}: hipBLASLt _int_mm {t_lt:7.1f} us ({f / t_lt / 1e6:5.0f} TOPS)  rocBLAS standard "
              f"{t_std:7.1f} us  best of {size.value} solutions {best[0][0]:7.1f} us ({f / best[0][0] / 1e6:5.0f} TOPS, "
              f"index {best[0][1]}; search {time.perf_counter() - t0:.1f} s; result ok {ok})", flush=True)
    rb.rocblas_destroy_handle(h)


if __name__ == "__main__":
    main()
