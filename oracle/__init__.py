"""CPU oracle for the quantized-matmul hot path — TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU, the algorithm the reference
(abhilash1910/bitsandbytes-SYCL, snapshot 2024-10-08) encodes for the hot path:
blockwise NF4/FP4/8-bit quantize + dequantize, the 4-bit GEMV/GEMM, the LLM.int8
row/col statistics, double_quant, the col32/col_turing/col_ampere layouts,
igemmlt and mm_dequant.  Every function cites the reference file:line it follows.

Who may use it: ONLY ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` — and there only as the checker / the timed
CPU baseline, never as the thing measured on the GPU or shipped.  The product
(``bitsandbytes-sycl_amd/python_src_quants``) never imports this package.

Parity pinning status:
  * the reference ships NO golden vectors / known-answer tests for this path and
    executing the reference (Python or C++) is not permitted in this pipeline
    (SURVEY.md §8c), so the oracle is pinned by the reference's *source
    constants* (NF4/FP4 tables and thresholds, MM_DEQUANT_CONST, layout index
    maps — cross-checked between the two places each one appears in the
    reference) and by the reference tests' tolerance contracts
    (tests_pvc/autograd.py:388-391, 277-280; test_matmulqlt.py:194-204).
    Quantize-index parity is therefore "partially pinned": pinned by source
    constants, not by reference-produced vectors.
"""
