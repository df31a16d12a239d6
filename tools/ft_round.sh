set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_matmul4bit_gpu.py -x -q -m gpu -k "fewtok" --timeout 120 --timeout-method thread > gpurun_out/ft_test.log 2>&1 || { tail -30 gpurun_out/ft_test.log; exit 1; }
tail -2 gpurun_out/ft_test.log
FT_SHAPES=11008x4096,4096x11008,4096x4096 FT_TOKENS=1,8,16,32 timeout -k 10 200 python -u tools/fewtok32_ab.py > gpurun_out/ft_ab.log 2>&1 || { tail -20 gpurun_out/ft_ab.log; exit 2; }
grep -v amdgpu.ids gpurun_out/ft_ab.log
for a in 0 1 4; do timeout -k 10 100 python -u tools/fewtok32_timeline.py 8 $a > gpurun_out/ft_tl8_$a.log 2>&1 || exit 3; done
cat gpurun_out/ft_tl8_*.log | grep -v amdgpu.ids
