#!/bin/bash
# Round 5: the k_hgemm timeline by physical XCD, then the full round (tools/gpu_round.sh).  Stops at the first failure.
# Usage (via gpurun, from the repo root): bash tools/r05d_session.sh <tag>
set -o pipefail
TAG=${1:-r05d}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u tools/hgemm_timeline.py > $OUT/${TAG}_hgemm_timeline.txt 2>&1 || { echo "timeline failed"; tail -20 $OUT/${TAG}_hgemm_timeline.txt; exit 1; }
grep -E "==|by blockIdx|by XCC|XCC_ID of" $OUT/${TAG}_hgemm_timeline.txt
bash tools/gpu_round.sh $TAG
