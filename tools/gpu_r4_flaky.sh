#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
cp tigerbeetle_amd/libtbgpu.so /tmp/keep.so
for v in N O N; do
  cp tigerbeetle_amd/libtbgpu_$v.so tigerbeetle_amd/libtbgpu.so
  timeout -k 10 200 python -u -m pytest tests/test_gpu_shard_surface.py -m gpu -q --timeout 150 --timeout-method thread -k "two_rank_gloo" > gpurun_out/r4/flaky_$v.log 2>&1; echo "$v rc=$?"; tail -1 gpurun_out/r4/flaky_$v.log
done
cp /tmp/keep.so tigerbeetle_amd/libtbgpu.so
