#!/bin/bash
# GPU side of tools/hgemm_plan_sweep.sh: every built plan variant at the metric shape, twice in alternating order.
set -o pipefail
mkdir -p gpurun_out
for pass in 1 2; do
  for b in tools/_bin/hgemm_lab_p*; do
    echo "== $(basename $b) pass $pass"
    timeout -k 10 60 $b 4096 4096 11008 5 || { echo "failed: $b"; exit 1; }
  done
done
