#!/bin/bash
# Round 5, one GPU-box session: the new features' GPU tests, then the A/B tool (epilogue, dequantise statistics, t64
# waves), then the bench's N-rank self-launch on the box's one GPU (gloo).  Stops at the first failure.
# Usage (via gpurun, from the repo root): bash tools/r05_ab_session.sh <tag>
set -o pipefail
TAG=${1:-r05a}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dequant_nested_gpu.py \
    tests/test_ipc_gpu.py tests/test_t64_gpu.py tests/test_prefetch_gpu.py tests/test_hgemm_gpu.py tests/test_configs_gpu.py \
    -k "nested_scalar or ipc or t64 or combine or prefetch or chunked or metric_shape or hgemm" > $OUT/${TAG}_tests.log 2>&1 \
    || { echo "tests failed"; tail -30 $OUT/${TAG}_tests.log; exit 1; }
tail -2 $OUT/${TAG}_tests.log
timeout -k 10 300 python -u tools/r05_epi_ab.py 5 > $OUT/${TAG}_ab.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/${TAG}_ab.txt; exit 2; }
cat $OUT/${TAG}_ab.txt
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --no-extras --steps 10 --warmup 3 > $OUT/${TAG}_bench2.json \
    2> $OUT/${TAG}_bench2.err || { echo "2-rank bench failed"; tail -20 $OUT/${TAG}_bench2.err; exit 3; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('2-rank bench:', d['n_gpus'], d['value'], d['config']['parallelism'])" $OUT/${TAG}_bench2.json
