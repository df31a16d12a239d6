#!/bin/bash
# Build GEMV variant libraries (round 6 A/B, CPU side): gemv4bit.hip with / without kernarg preloading
# (-mllvm -amdgpu-kernarg-preload-count=16) x the weights issued before / after the statistics (-DBNB_GV_WFIRST),
# every other object from the product build.  Output: tools/_lab/libbnb_gv_kp{0,1}_wf{0,1}.so
set -e
cd "$(dirname "$0")/../bitsandbytes-sycl_amd/csrc"
make -j8 >/dev/null
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-result -Wno-unused-value -ffp-contract=off"
OBJS=$(ls ../build/obj/*.o | grep -v "/gemv4bit.o$")
mkdir -p ../build/objgv ../../tools/_lab
for kp in 0 1; do for wf in 0 1; do
  X=""; [ $kp = 1 ] && X="-mllvm -amdgpu-kernarg-preload-count=16"
  /opt/rocm/bin/hipcc $F $X -DBNB_GV_WFIRST=$wf -c gemv4bit.hip -o ../build/objgv/gemv_kp${kp}_wf${wf}.o &
done; done
wait
for kp in 0 1; do for wf in 0 1; do
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS ../build/objgv/gemv_kp${kp}_wf${wf}.o -pthread -lrocblas \
    -o ../../tools/_lab/libbnb_gv_kp${kp}_wf${wf}.so
done; done
ls -la ../../tools/_lab/
