#!/bin/bash
# PMC passes over a lab binary (each pass its own process; --pmc never combined with tracing).
# Usage: bash tools/lab_counters.sh <tag> <binary> [args...]
TAG=$1; shift
OUT=gpurun_out/lab_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for SET in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA" \
           "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM" \
           "GRBM_GUI_ACTIVE SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $SET --output-format csv -d $OUT/p$i -- "$@" > $OUT/p$i.log 2>&1
  echo "pass $i rc=$?" >> $OUT/status.txt
done
python3 tools/lab_summary.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
