#!/bin/bash
# Build a compile-time variant of the product library for an A/B run:
#   scripts/build_variant.sh NAME "-DMACRO=VALUE ..."  ->  chunker_amd/_ab/libchunker_amd_NAME.so
# (load it with CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_NAME.so)
set -e
cd "$(dirname "$0")/../chunker_amd/csrc"
make -s -j8 OBJDIR=_obj_$1 OUT=../_ab/libchunker_amd_$1.so \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $2" ../_ab/libchunker_amd_$1.so
