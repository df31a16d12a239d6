#!/bin/bash
# Round 6: prefetch tests (both side forms), the hgemm determinism test, then the tail-form A/B.
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_prefetch_gpu.py tests/test_hgemm_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/r06c_tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/r06c_tests.log; exit 1; }
tail -2 $OUT/r06c_tests.log
timeout -k 10 400 python tools/r06_tail_ab.py > $OUT/r06c_tail_ab.json 2> $OUT/r06c_tail_ab.err || { echo "ab failed"; tail -20 $OUT/r06c_tail_ab.err; exit 2; }
cat $OUT/r06c_tail_ab.json
