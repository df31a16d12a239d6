set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/pmc_ft
for M in 1 8; do
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/pmc_ft/tr$M -- python3 tools/fewtok32_probe.py 2 $M > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/pmc_ft/f$M -- python3 tools/fewtok32_probe.py 2 $M > /dev/null 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T --output-format csv -d gpurun_out/pmc_ft/h$M -- python3 tools/fewtok32_probe.py 2 $M > /dev/null 2>&1 || exit 3
done
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/pmc_ft/fgemv -- python3 tools/fewtok32_probe.py 1 8 > /dev/null 2>&1 || exit 4
echo ok
