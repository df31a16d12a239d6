#!/bin/bash
# GPU side of the round-6 kernel-argument-preload A/B: the few-token kernels' variant library against the base
# (product) library, 4 interleaved rounds, one process per run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/kp_fewtok.jsonl
for r in 1 2 3 4; do
  for v in base kpft; do
    BNB_HIP_LIBRARY=$PWD/tools/_lab/libbnb_$v.so timeout -k 10 150 python -u tools/r06_fewtok_variant_time.py \
      >> gpurun_out/kp_fewtok.jsonl 2> gpurun_out/kp_err.log || { cat gpurun_out/kp_err.log; exit 1; }
  done
done
cat gpurun_out/kp_fewtok.jsonl
