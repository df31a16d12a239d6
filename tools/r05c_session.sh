#!/bin/bash
# Round 5: the register-fed 33..64-token form -- its GPU tests (t64 file), then the A/B timing.  Stops at the first failure.
# Usage (via gpurun, from the repo root): bash tools/r05c_session.sh <tag>
set -o pipefail
TAG=${1:-r05c}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_t64_gpu.py -k "t64r" \
    > $OUT/${TAG}_t64r_tests.log 2>&1 || { echo "t64r tests failed"; tail -40 $OUT/${TAG}_t64r_tests.log; exit 1; }
tail -2 $OUT/${TAG}_t64r_tests.log
timeout -k 10 300 python -u tools/r05_t64r_ab.py 5 > $OUT/${TAG}_t64r_ab.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/${TAG}_t64r_ab.txt; exit 2; }
cat $OUT/${TAG}_t64r_ab.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_t64_gpu.py \
    > $OUT/${TAG}_t64_tests.log 2>&1 || { echo "t64 tests failed"; tail -40 $OUT/${TAG}_t64_tests.log; exit 3; }
tail -2 $OUT/${TAG}_t64_tests.log
