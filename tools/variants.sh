#!/bin/bash
# Builds A/B variants of libtbgpu.so: tools/variants.sh NAME "-DFLAG=V ..." [NAME "flags"]...
# (tigerbeetle_amd/libtbgpu_NAME.so, same sources and flags as build.py plus the given defines)
cd "$(dirname "$0")/../tigerbeetle_amd" || exit 1
while [ $# -ge 2 ]; do
  hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -Wall $2 -o libtbgpu_$1.so \
    csrc/engine.hip csrc/workload.hip csrc/checksum.hip || exit 1
  shift 2
done
