set -o pipefail
mkdir -p gpurun_out
FT_SHAPES=11008x4096,4096x4096 FT_TOKENS=1,8 timeout -k 10 200 python -u tools/fewtok32_ab.py 256 260 > gpurun_out/ft_rw_ab.log 2>&1 || { tail -20 gpurun_out/ft_rw_ab.log; exit 2; }
grep -v amdgpu.ids gpurun_out/ft_rw_ab.log
timeout -k 10 100 python -u tools/fewtok32_timeline.py 8 256 > gpurun_out/ft_tl_rw.log 2>&1 || exit 3
cat gpurun_out/ft_tl_rw.log | grep -v amdgpu.ids
