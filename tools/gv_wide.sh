set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_matmul4bit_gpu.py -x -q -m gpu -k "gemv_wide or gemv" --timeout 120 --timeout-method thread > gpurun_out/gv_test.log 2>&1 || { tail -30 gpurun_out/gv_test.log; exit 1; }
tail -2 gpurun_out/gv_test.log
timeout -k 10 150 python -u tools/decode70_probe.py > gpurun_out/decode70b.log 2>&1 || exit 4
grep -v amdgpu.ids gpurun_out/decode70b.log
