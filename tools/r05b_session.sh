#!/bin/bash
# Round 5, second GPU session: the MFMA + decode-VALU issue lab, the C-store non-temporal A/B, then the full round
# (tools/gpu_round.sh: GPU tests, smoke, bench, rocprofv3).  Stops at the first failure.
# Usage (via gpurun, from the repo root): bash tools/r05b_session.sh <tag>
set -o pipefail
TAG=${1:-r05b}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 120 tools/_bin/mfma_valu_mix_lab > $OUT/${TAG}_mix.txt 2>&1 || { echo "mix lab failed"; cat $OUT/${TAG}_mix.txt; exit 1; }
cat $OUT/${TAG}_mix.txt
timeout -k 10 300 python -u tools/r05_cstore_ab.py 7 > $OUT/${TAG}_cstore.txt 2>&1 || { echo "cstore ab failed"; tail -20 $OUT/${TAG}_cstore.txt; exit 2; }
cat $OUT/${TAG}_cstore.txt
bash tools/gpu_round.sh $TAG
