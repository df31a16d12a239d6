#!/bin/bash
# Build a lab binary with its ISA next to it: bash tools/labbuild.sh gemm_lab2
set -e -o pipefail
cd "$(dirname "$0")/.."
mkdir -p tools/_bin
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off ${LABFLAGS--fno-slp-vectorize} -Wno-unused-result -I bitsandbytes-sycl_amd/csrc -I tools tools/$1.hip -o tools/_bin/$1 --save-temps=obj 2>&1 | grep -E "error|Error" || true
