#!/bin/bash
# Device assembly of one SpMM translation unit at the headline shape only (r = 5, d = 3), for inspecting
# a kernel's loop schedule / registers:  tools/isa_dump.sh <TU 1..5> <out.s>
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DDPGO_ISA_54_ONLY -DDPGO_SPMM_TU="$1" $ISA_FLAGS --cuda-device-only -S \
  -Iinclude -o "$2" dpgo_amd/csrc/kernels.hip
