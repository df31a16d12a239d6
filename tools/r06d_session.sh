#!/bin/bash
# Round 6 validation, part 1: the full -m gpu suite, smoke(), the tail-form A/B.
set -o pipefail
TAG=${1:-r06d}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 $OUT/gpu_tests_$TAG.log; exit 1; }
tail -2 $OUT/gpu_tests_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke_$TAG.log; exit 2; }
tail -1 $OUT/smoke_$TAG.log
timeout -k 10 200 python tools/r06_tail_ab.py > $OUT/${TAG}_tail_ab.json 2> $OUT/${TAG}_tail_ab.err || { echo "ab failed"; tail -20 $OUT/${TAG}_tail_ab.err; exit 3; }
cat $OUT/${TAG}_tail_ab.json
