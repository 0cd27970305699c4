mkdir -p gpurun_out/v6
cp tigerbeetle_amd/libtbgpu.so /tmp/libtbgpu.keep.so && cp tigerbeetle_amd/libtbgpu_prof.so tigerbeetle_amd/libtbgpu.so
timeout -k 10 120 python tools/cfg3_probe.py 6 32 > gpurun_out/v6/probe.log 2>&1
cp /tmp/libtbgpu.keep.so tigerbeetle_amd/libtbgpu.so
