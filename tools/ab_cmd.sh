#!/bin/bash
# A/B of library builds on one box for any command: VARIANTS="A B" tools/ab_cmd.sh ROUNDS CMD...
# (copies tigerbeetle_amd/libtbgpu_<v>.so over libtbgpu.so in turn, runs CMD under a time limit, keeps
# its last stdout line per run in gpurun_out/ab/<v>_<round>.log; the tree's library is restored on exit).
n=$1; shift
mkdir -p gpurun_out/ab
cp tigerbeetle_amd/libtbgpu.so /tmp/libtbgpu.keep.so
trap 'cp /tmp/libtbgpu.keep.so tigerbeetle_amd/libtbgpu.so' EXIT
for r in $(seq 1 "$n"); do
  for v in ${VARIANTS:-A B}; do
    cp tigerbeetle_amd/libtbgpu_$v.so tigerbeetle_amd/libtbgpu.so
    timeout -k 10 300 "$@" > gpurun_out/ab/${v}_$r.log 2> gpurun_out/ab/${v}_$r.err || { echo "$v failed"; tail -3 gpurun_out/ab/${v}_$r.err; exit 1; }
    echo "$v $r $(tail -c 400 gpurun_out/ab/${v}_$r.log)"
  done
done
