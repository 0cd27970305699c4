#!/bin/bash
# A/B timing of builds of libtbgpu.so on one box: VARIANTS="A B" tools/ab.sh <config> <rounds> [bench args]
# (copies tigerbeetle_amd/libtbgpu_<v>.so over libtbgpu.so in turn; results in gpurun_out/ab_*.log).
# The tree's own library is restored on every exit path.
cfg=$1; n=$2; shift 2
cp tigerbeetle_amd/libtbgpu.so /tmp/libtbgpu.keep.so
trap 'cp /tmp/libtbgpu.keep.so tigerbeetle_amd/libtbgpu.so' EXIT
for r in $(seq 1 "$n"); do
  for v in ${VARIANTS:-A B}; do
    cp tigerbeetle_amd/libtbgpu_$v.so tigerbeetle_amd/libtbgpu.so
    timeout -k 10 180 python bench.py --config "$cfg" --no-cpu-baseline --host-fed-transfers 0 --sync-commit-batches 0 "$@" > gpurun_out/ab_${cfg}_${v}_$r.log 2>&1 || exit 1
    python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['value'],d['roofline'].get('phase_avg_us_warmup'))" gpurun_out/ab_${cfg}_${v}_$r.log $v
  done
done
