#!/bin/bash
# Round 6 GPU session: the full -m gpu suite, smoke(), the default bench (one box, one call).
set -o pipefail
TAG=${1:-r06b}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 $OUT/gpu_tests_$TAG.log; exit 1; }
tail -2 $OUT/gpu_tests_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke_$TAG.log; exit 2; }
tail -1 $OUT/smoke_$TAG.log
timeout -k 10 400 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed"; tail -20 $OUT/bench_$TAG.err; exit 3; }
cat $OUT/bench_$TAG.json
