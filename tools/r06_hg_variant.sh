#!/bin/bash
# Build a variant of the product library with hgemm.hip compiled with extra flags (round 6 A/B):
#   tools/r06_hg_variant.sh <name> <flags...>  ->  tools/_lab/libbnb_<name>.so
set -e
name=$1; shift
cd "$(dirname "$0")/../bitsandbytes-sycl_amd/csrc"
make -j8 >/dev/null
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-result -Wno-unused-value -ffp-contract=off"
mkdir -p ../build/objhg ../../tools/_lab
/opt/rocm/bin/hipcc $F "$@" -c hgemm.hip -o ../build/objhg/hgemm_$name.o
OBJS=$(ls ../build/obj/*.o | grep -v "/hgemm.o$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS ../build/objhg/hgemm_$name.o -pthread -lrocblas \
  -o ../../tools/_lab/libbnb_$name.so
ls -la ../../tools/_lab/libbnb_$name.so
