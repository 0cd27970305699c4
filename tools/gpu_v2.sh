# chunked resolver: resolver/limit parity tests, cfg3 bench, kernel trace and probe (RC_PROF build)
mkdir -p gpurun_out/v2
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_resolver.py tests/test_gpu_bind.py tests/test_gpu_geometry.py tests/test_gpu_configs.py tests/test_gpu_kat.py -x -v --timeout 200 --timeout-method thread > gpurun_out/v2/pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config cfg3 --no-cpu-baseline --host-fed-transfers 0 > gpurun_out/v2/bench_cfg3.json 2> gpurun_out/v2/bench_cfg3.err || exit 1
true
cp tigerbeetle_amd/libtbgpu.so /tmp/libtbgpu.keep.so && cp tigerbeetle_amd/libtbgpu_prof.so tigerbeetle_amd/libtbgpu.so
timeout -k 10 120 python tools/cfg3_probe.py 6 32 > gpurun_out/v2/probe.log 2>&1
cp /tmp/libtbgpu.keep.so tigerbeetle_amd/libtbgpu.so
