#!/bin/bash
# Round 6: per-wave timeline of the few-token kernel at 8 and 32 tokens, and the 32-token ablations (lab build)
set -o pipefail
mkdir -p gpurun_out
export BNB_HIP_LIBRARY=$PWD/tools/_lab/libbitsandbytes_hip_lab.so
out=gpurun_out/fewtok32_tl.txt
: > $out
for args in "8 0" "32 0" "32 1" "32 4" "32 2" "32 7"; do
  timeout -k 10 120 python -u tools/fewtok32_timeline.py $args >> $out 2>gpurun_out/fewtok32_tl.err || { cat gpurun_out/fewtok32_tl.err; exit 1; }
done
cat $out
