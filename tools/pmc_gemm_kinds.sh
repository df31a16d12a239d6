# PMC passes (MFMA busy, clock) for the three GEMM kinds at 4096 x 4096 x 11008 (tools/gemm_kind_probe.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/pmc_kinds
mkdir -p $OUT
for K in i8_8w i8_4w bf16; do
  timeout -k 10 120 python3 tools/gemm_kind_probe.py $K >> $OUT/times.txt 2>/dev/null || exit 1
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -T --output-format csv -d $OUT/$K -- python3 tools/gemm_kind_probe.py $K > /dev/null 2>&1 || exit 2
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA -T --output-format csv -d $OUT/${K}_w -- python3 tools/gemm_kind_probe.py $K > /dev/null 2>&1 || exit 3
done
cat $OUT/times.txt
