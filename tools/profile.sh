#!/bin/bash
# Profile the bench on the GPU box: kernel trace + stats, then two PMC passes (FETCH_SIZE, WRITE_SIZE).
# Usage (from the repo root, via gpurun): bash tools/profile.sh <tag>
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT profiles
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
# the metric step alone (its kernel means must agree with the bench's event times), then the extra legs
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extras > $OUT/bench_traced.json 2> $OUT/trace.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace_extras -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $OUT/bench_traced_extras.json 2> $OUT/trace_extras.err || exit 5
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/fetch -- python3 bench.py --no-extras --no-cpu --steps 3 --warmup 1 > /dev/null 2> $OUT/fetch.err || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/write -- python3 bench.py --no-extras --no-cpu --steps 3 --warmup 1 > /dev/null 2> $OUT/write.err || exit 3
# MFMA utilisation and the clock held under load (counters only; durations come from the trace pass above)
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -T --output-format csv -d $OUT/mfma -- python3 bench.py --no-extras --no-cpu --steps 3 --warmup 1 > /dev/null 2> $OUT/mfma.err || exit 6
# the kernel that carries the metric's flops at 4096 x 4096 x 11008 (bench.gemm_kernel_name): the library
# GEMM (Cijk_*) after the dequantise kernel, or the fused k_gemm_4bit_256 when routed there
LABEL=$(python3 -c "import bench; print(bench.gemm_kernel_name(4096, 4096))" 2>/dev/null | tail -1)
# library route: the exact name of the most-launched Cijk kernel of the metric trace (the per-shape solution search
# launches other Cijk kernels a few times each on the first call; a substring match would count them too)
case "$LABEL" in
  library*) MATCH=$(python3 -c "
import csv, glob, sys
rows = [r for p in glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True) for r in csv.DictReader(open(p))
        if 'Cijk' in r['Name']]
print(max(rows, key=lambda r: int(r['Calls']))['Name'] if rows else 'Cijk')" $OUT/trace) ;;
  k_hgemm*) MATCH="k_hgemm" ;;
  *) MATCH="k_gemm_4bit_256" ;;
esac
python3 tools/pmc_traffic.py $OUT/fetch $OUT/write "$MATCH" $OUT/pmc_traffic.json 4096 4096 11008 "$LABEL" $OUT/mfma $OUT/trace || exit 4
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/${TAG}_kernel_stats.csv \;
find $OUT/trace_extras -name "*kernel_stats.csv" -exec cp {} $OUT/${TAG}_kernel_stats_extras.csv \;
echo "profile done"
