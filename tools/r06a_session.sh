set -o pipefail
OUT=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ipc_gpu.py tests/test_rccl_gpu.py -x -v --timeout 200 --timeout-method thread > $OUT/r06a_tests.log 2>&1 || { echo tests failed; tail -30 $OUT/r06a_tests.log; exit 1; }
tail -3 $OUT/r06a_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras > $OUT/r06a_bench1.json 2> $OUT/r06a_bench1.err || { echo bench1 failed; tail -20 $OUT/r06a_bench1.err; exit 2; }
cat $OUT/r06a_bench1.json
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-extras > $OUT/r06a_bench2.json 2> $OUT/r06a_bench2.err || { echo bench2 failed; tail -30 $OUT/r06a_bench2.err; exit 3; }
cat $OUT/r06a_bench2.json
