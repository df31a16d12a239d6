#!/bin/bash
# Round 6 validation, part 2: the default bench, then the rocprofv3 profile of the metric step (tools/profile.sh).
set -o pipefail
TAG=${1:-r06e}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 420 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed"; tail -20 $OUT/bench_$TAG.err; exit 3; }
cat $OUT/bench_$TAG.json
bash tools/profile.sh $TAG || { echo "profile failed"; exit 4; }
