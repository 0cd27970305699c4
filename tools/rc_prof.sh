# cfg3 with the RC_PROF=1 library (per-phase cycles of k_rc_run into the debug counters)
cp tigerbeetle_amd/libtbgpu.so /tmp/libtbgpu.keep.so
trap 'cp /tmp/libtbgpu.keep.so tigerbeetle_amd/libtbgpu.so' EXIT
cp tigerbeetle_amd/libtbgpu_P.so tigerbeetle_amd/libtbgpu.so
mkdir -p gpurun_out/p
TBG_DEBUG=1 timeout -k 10 300 python bench.py --config cfg3 --no-cpu-baseline --host-fed-transfers 0 > gpurun_out/p/cfg3.json 2> gpurun_out/p/cfg3.err
grep "resolver counters" gpurun_out/p/cfg3.err
