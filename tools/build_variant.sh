#!/bin/bash
# Build a variant of the engine library for tools/exp_ab_libs.py:
#   tools/build_variant.sh NAME [extra hipcc flags...]  ->  build/ab/NAME/libhadoofus_crc32c.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
OUT=${AB_OUT:-$ROOT/build/ab}/$NAME
mkdir -p "$OUT"
C=$ROOT/hadoofus_amd/csrc
# same flags as hadoofus_amd/build.py (pass extra ones after NAME)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-function \
  -mllvm -amdgpu-atomic-optimizer-strategy=None \
  -Wl,--version-script=$C/exports.map -I$ROOT/include -I$C "$@" -o "$OUT/libhadoofus_crc32c.so" \
  $C/crc32c_kernels.hip $C/crc32c_probes.hip $C/crc32c_engine.cpp $C/crc32c_packets.cpp
echo "$OUT/libhadoofus_crc32c.so"
