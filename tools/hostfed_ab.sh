#!/bin/bash
# Host-fed rate (bench.py cfg2 `host_fed`) for builds of libtbgpu.so: VARIANTS="A B" tools/hostfed_ab.sh <rounds>
# (A with HSA_ENABLE_SDMA=0 as variant "A0"); results in gpurun_out/hf/.
n=${1:-2}; shift
mkdir -p gpurun_out/hf
cp tigerbeetle_amd/libtbgpu.so /tmp/libtbgpu.keep.so
trap 'cp /tmp/libtbgpu.keep.so tigerbeetle_amd/libtbgpu.so' EXIT
for r in $(seq 1 "$n"); do
  for v in ${VARIANTS:-A B}; do
    lib=${v%0}
    cp tigerbeetle_amd/libtbgpu_$lib.so tigerbeetle_amd/libtbgpu.so
    if [ "$v" != "$lib" ]; then export HSA_ENABLE_SDMA=0; else unset HSA_ENABLE_SDMA; fi
    timeout -k 10 200 python bench.py --config cfg2 --no-cpu-baseline --no-phase-timing "$@" > gpurun_out/hf/${v}_$r.json 2> gpurun_out/hf/${v}_$r.err || exit 1
    python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);h=d['host_fed'];print(sys.argv[2],d['value'],h['value'],h['h2d_GBs'])" gpurun_out/hf/${v}_$r.json $v
  done
done
