#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench (default args), rocprofv3 profile.  Stops at the first failure.
# Usage (via gpurun, from the repo root): bash tools/gpu_round.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out
mkdir -p $OUT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -30 $OUT/gpu_tests_$TAG.log; exit 1; }
  tail -2 $OUT/gpu_tests_$TAG.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke_$TAG.log; exit 2; }
  tail -1 $OUT/smoke_$TAG.log
fi
timeout -k 10 400 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed"; tail -20 $OUT/bench_$TAG.err; exit 3; }
cat $OUT/bench_$TAG.json
bash tools/profile.sh $TAG || { echo "profile failed"; exit 4; }
