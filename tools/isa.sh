#!/bin/bash
# Dump gfx950 assembly of one translation unit (default: the SimpleReacher episode kernels).
cd "$(dirname "$0")/.."
SRC=${1:-fgx_ep_simple.hip}
OUT=${2:-/tmp/isa/$(basename "$SRC" .hip).s}
mkdir -p "$(dirname "$OUT")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -Wno-unused-result -I include \
  --cuda-device-only -S fancy_gym_crowd_amd/csrc/$SRC -o "$OUT" && echo "$OUT"
