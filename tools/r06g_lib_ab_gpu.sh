#!/bin/bash
# Interleaved A/B of library builds on the GPU box (round 6): bash tools/r06g_lib_ab_gpu.sh <timing script> <out> <lib>...
# runs the timing script once per library per round (4 rounds, one process each), appending its JSON lines to <out>.
set -o pipefail
script=$1; out=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
: > $out
for r in 1 2 3 4; do
  for lib in "$@"; do
    BNB_HIP_LIBRARY=$PWD/$lib timeout -k 10 150 python -u $script >> $out 2> gpurun_out/lib_ab_err.log \
      || { cat gpurun_out/lib_ab_err.log; exit 1; }
  done
done
cat $out
