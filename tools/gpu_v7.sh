# A/B of the chunked resolver's wave walker: one vs two entries per lane (probe + tests + cfg3 bench)
mkdir -p gpurun_out/v7
cp tigerbeetle_amd/libtbgpu.so /tmp/keep.so
for v in prof prof2; do
  cp tigerbeetle_amd/libtbgpu_$v.so tigerbeetle_amd/libtbgpu.so
  timeout -k 10 120 python tools/cfg3_probe.py 6 32 > gpurun_out/v7/probe_$v.log 2>&1 || break
done
cp tigerbeetle_amd/libtbgpu_x2.so tigerbeetle_amd/libtbgpu.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_resolver.py tests/test_gpu_bind.py tests/test_gpu_geometry.py -x -q --timeout 200 --timeout-method thread > gpurun_out/v7/pytest_x2.log 2>&1 && \
timeout -k 10 200 python bench.py --config cfg3 --no-cpu-baseline --host-fed-transfers 0 > gpurun_out/v7/bench_cfg3_x2.json 2> gpurun_out/v7/bench_cfg3_x2.err
cp /tmp/keep.so tigerbeetle_amd/libtbgpu.so
