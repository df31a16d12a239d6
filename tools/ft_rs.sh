set -o pipefail
mkdir -p gpurun_out
FT_SHAPES=11008x4096,4096x11008 FT_TOKENS=1,8 timeout -k 10 200 python -u tools/fewtok32_ab.py 512 > gpurun_out/ft_rs_ab.log 2>&1 || { tail -20 gpurun_out/ft_rs_ab.log; exit 2; }
grep -v amdgpu.ids gpurun_out/ft_rs_ab.log
timeout -k 10 100 python -u tools/fewtok32_timeline.py 8 512 > gpurun_out/ft_tl_rs.log 2>&1 || exit 3
grep -v amdgpu.ids gpurun_out/ft_tl_rs.log
timeout -k 10 150 python -u tools/decode70_probe.py > gpurun_out/decode70.log 2>&1 || exit 4
grep -v amdgpu.ids gpurun_out/decode70.log
