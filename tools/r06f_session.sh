#!/bin/bash
# Round 6: the default bench at HEAD (sampled step events, int8 leg without events), then the 2-rank gloo rehearsal.
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 420 python bench.py > $OUT/bench_r06f.json 2> $OUT/bench_r06f.err || { echo "bench failed"; tail -20 $OUT/bench_r06f.err; exit 1; }
cat $OUT/bench_r06f.json
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-extras > $OUT/bench_r06f_n2.json 2> $OUT/bench_r06f_n2.err || { echo "bench2 failed"; tail -30 $OUT/bench_r06f_n2.err; exit 2; }
cat $OUT/bench_r06f_n2.json
