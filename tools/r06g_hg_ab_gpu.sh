#!/bin/bash
# Round 6: hgemm.hip variant A/B on the GPU box -- the variant library through the k_hgemm / int8 / fuzz tests, then 4
# interleaved rounds of tools/r06_hg_variant_time.py on the base and the variant library.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$1
BNB_HIP_LIBRARY=$PWD/tools/_lab/libbnb_$V.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_hgemm_gpu.py tests/test_int8_gpu.py tests/test_fuzz_gpu.py > gpurun_out/hg_ab_tests_$V.log 2>&1 \
  || { tail -30 gpurun_out/hg_ab_tests_$V.log; exit 1; }
tail -1 gpurun_out/hg_ab_tests_$V.log
bash tools/r06g_lib_ab_gpu.sh tools/r06_hg_variant_time.py gpurun_out/hg_ab_$V.jsonl tools/_lab/libbnb_hgbase.so tools/_lab/libbnb_$V.so
