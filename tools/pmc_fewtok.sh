#!/bin/bash
# PMC HBM traffic of the decode GEMV and few-token kernels (bench legs), one counter block per pass.
# Usage (via gpurun, from the repo root): bash tools/pmc_fewtok.sh <tag>
set -o pipefail
TAG=${1:-r05}
OUT=gpurun_out/pmc_fewtok_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/fetch -- python3 tools/pmc_fewtok_legs.py > $OUT/legs_fetch.txt 2> $OUT/fetch.err || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/write -- python3 tools/pmc_fewtok_legs.py > $OUT/legs_write.txt 2> $OUT/write.err || exit 2
python3 tools/pmc_fewtok_summary.py $OUT/fetch $OUT/write > $OUT/summary.txt || exit 3
cat $OUT/summary.txt
