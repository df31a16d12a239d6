#!/bin/bash
# Build hgemm_lab with the (8, 8) three-barrier plan's barriers moved (HgPlan3<8, 8>: HG_P3_DB1 / DB2 / DB3 shift B1 / B2
# / B3 and the fragment reads / DMA pieces keyed to each), one binary per variant: tools/_bin/hgemm_lab_p<d1>_<d2>_<d3>.
# A fifth field sets HG_P3_AEARLY (the last 3 A pieces before B3).  A fourth field sets HG_P3_ABL (lab ablation: 1 = no barrier at B1 / B2, 2 = no lgkmcnt wait there; timing only).
# Usage: bash tools/hgemm_plan_sweep.sh "0,0,0 3,0,0 0,0,0,1 ..."   (run each binary on the GPU box: tools/_bin/hgemm_lab_p...)
set -e -o pipefail
cd "$(dirname "$0")/.."
mkdir -p tools/_bin
for v in $1; do
  IFS=, read -r d1 d2 d3 abl ae <<< "$v"
  abl=${abl:-0}
  ae=${ae:-0}
  tag="p${d1}_${d2}_${d3}_a${abl}_e${ae}"
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -Wno-unused-result \
      -DHG_P3_DB1=$d1 -DHG_P3_DB2=$d2 -DHG_P3_DB3=$d3 -DHG_P3_ABL=$abl -DHG_P3_AEARLY=$ae -I bitsandbytes-sycl_amd/csrc -I tools tools/hgemm_lab.hip \
      -o tools/_bin/hgemm_lab_$tag -lrocblas 2>&1 | grep -E "error" ; true ) &
  while [ "$(jobs -r | wc -l)" -ge 4 ]; do sleep 2; done
done
wait
ls tools/_bin/ | grep hgemm_lab_p
