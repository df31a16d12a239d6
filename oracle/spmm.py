"""numpy restatement of the reference's COO sparse x dense products (TEST INFRASTRUCTURE ONLY; see
oracle/__init__.py for who may import this).

  spmm_coo_very_sparse   ref:sycl/sycl_code/kernel_gemm.cpp:1398-1545 (kspmm_coo_very_sparse_naive),
                         wrapper ref:python_src_quants/functional.py:2704-2782
  spmm_coo               ref:python_src_quants/functional.py:2656-2701 -> cspmm_coo, which the reference
                         leaves commented out (pythonInterface.cpp:358-361, Q18); restated as the upstream
                         cuSPARSE SpMM it wraps: C = A @ B, fp32 accumulation, beta = 0

Parity: unpinned by any reference run or fixture (the reference ships none for these kernels); the
restatement follows the kernel source expression by expression (fp16 accumulator rounded after every
nonzero, in-place fp16 update of `out`).
"""
from __future__ import annotations

import numpy as np

F16 = np.float16
F32 = np.float32


def very_sparse_launch_args(rowidx: np.ndarray):
    """The wrapper's preprocessing (functional.py:2719-2724): row groups, their counts sorted descending,
    the group order and the cumulative offsets."""
    values, counts = np.unique(rowidx, return_counts=True)
    offset = np.cumsum(counts).astype(np.int32)
    order = np.argsort(-counts, kind="stable")
    return counts[order].astype(np.int32), order.astype(np.int32), offset, int(values.size)


def spmm_coo_very_sparse(rowidx, colidx, values, B, out, dequant_stats=None):
    """out (fp16 [rowsA, colsB]) updated in place and returned.  B: fp16 or int8 [rowsB, colsB]."""
    max_count, max_idx, offset, nnz_rows = very_sparse_launch_args(rowidx)
    out = out.astype(F16).copy()
    colsB = B.shape[1]
    denorm = F32(1.0) / F32(127.0)
    st = None
    if B.dtype == np.int8 and dequant_stats is not None:
        st = (np.asarray(dequant_stats, F32).astype(F16).astype(F32) * denorm).astype(F32)
    for b in range(nnz_rows):
        count = int(max_count[b])
        g = int(max_idx[b])
        off = 0 if g == 0 else int(offset[g - 1])
        row = int(rowidx[off])
        acc = np.zeros(colsB, F16)
        for i in range(count):
            a = F32(np.float16(values[off + i]))
            brow = B[int(colidx[off + i])].astype(F32)
            if st is not None:
                prod = ((st * brow).astype(F32) * a).astype(F32)
                upd = (acc.astype(F32) + prod).astype(F32).astype(F16)
                acc = np.where((brow != 0) & (a != 0), upd, acc)
            else:
                acc = (acc.astype(F32) + (brow * a).astype(F32)).astype(F32).astype(F16)
        out[row] = (out[row].astype(F32) + acc.astype(F32)).astype(F32).astype(F16)
    return out


def spmm_coo(rowidx, colidx, values, rows, B):
    """C = A @ B with fp32 accumulation in row-sorted nonzero order, one fp16 rounding."""
    order = np.argsort(rowidx, kind="stable")
    C = np.zeros((rows, B.shape[1]), F32)
    Bf = B.astype(F32)
    for e in order:
        C[int(rowidx[e])] = (C[int(rowidx[e])] + (F32(np.float16(values[e])) * Bf[int(colidx[e])]).astype(F32)).astype(F32)
    return C.astype(F16)
