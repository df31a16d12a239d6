#!/bin/bash
# Build a variant of the product library with kernel-argument preloading on the listed sources (round 6 A/B):
#   tools/r06_kp_variant.sh <name> <file.hip>...  ->  tools/_lab/libbnb_<name>.so
# Each listed file keeps its own Makefile flags (mirrored here) plus -mllvm -amdgpu-kernarg-preload-count=16.
set -e
name=$1; shift
cd "$(dirname "$0")/../bitsandbytes-sycl_amd/csrc"
make -j8 >/dev/null
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-result -Wno-unused-value -ffp-contract=off"
KP="-mllvm -amdgpu-kernarg-preload-count=16"
mkdir -p ../build/objkp/$name ../../tools/_lab
OBJS=""
for o in ../build/obj/*.o; do
  b=$(basename $o .o); skip=0
  for f in "$@"; do [ "$b" = "$(basename $f .hip)" ] && skip=1; done
  [ $skip = 0 ] && OBJS="$OBJS $o"
done
for f in "$@"; do
  X=""
  case $f in
    gemm4bit_fewtok.hip) X="-fno-slp-vectorize" ;;
    gemm4bit_t64.hip) X="-fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form=1" ;;
  esac
  /opt/rocm/bin/hipcc $F $X $KP -c $f -o ../build/objkp/$name/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS ../build/objkp/$name/*.o -pthread -lrocblas \
  -o ../../tools/_lab/libbnb_$name.so
ls -la ../../tools/_lab/libbnb_$name.so
