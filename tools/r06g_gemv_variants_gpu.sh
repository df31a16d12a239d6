#!/bin/bash
# GPU side of the round-6 GEMV variant A/B: GEMV tests on the product library, then 4 interleaved rounds of the four
# variant libraries (tools/r06_gemv_variants.sh), one process each.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_matmul4bit_gpu.py -k gemv \
  > gpurun_out/gv_tests.log 2>&1 || { tail -20 gpurun_out/gv_tests.log; exit 1; }
tail -1 gpurun_out/gv_tests.log
: > gpurun_out/gv_variants.jsonl
for r in 1 2 3 4; do
  for v in kp0_wf0 kp1_wf0 kp0_wf1 kp1_wf1; do
    BNB_HIP_LIBRARY=$PWD/tools/_lab/libbnb_gv_$v.so timeout -k 10 120 python -u tools/r06_gemv_variant_time.py \
      >> gpurun_out/gv_variants.jsonl 2> gpurun_out/gv_variant_err.log || { cat gpurun_out/gv_variant_err.log; exit 1; }
  done
done
cat gpurun_out/gv_variants.jsonl
