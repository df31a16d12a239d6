#!/bin/bash
# PMC passes on one kernel driver run (each pass its own process; --pmc never combined with tracing).
# Usage: bash tools/counters.sh <tag> <driver-args...>
TAG=$1; shift
OUT=gpurun_out/ctr_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for SET in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_INSTS_MFMA SQ_LDS_UNALIGNED_STALL SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $SET -T --output-format csv -d $OUT/p$i -- python3 tools/kernel_driver.py "$@" > $OUT/p$i.log 2>&1
  echo "pass $i rc=$?" >> $OUT/status.txt
done
timeout -k 10 120 python3 tools/kernel_driver.py "$@" > $OUT/plain.log 2>&1
echo done
