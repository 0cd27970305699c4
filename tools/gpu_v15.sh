# chunked-resolver parts: limit-path parity on the current build (E) and on F, then cfg3 A/B of D E F
mkdir -p gpurun_out/v15
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_resolver.py tests/test_gpu_bind.py tests/test_gpu_configs.py tests/test_gpu_geometry.py -x -q --timeout 200 --timeout-method thread > gpurun_out/v15/pytest_E.log 2>&1 || exit 1
cp tigerbeetle_amd/libtbgpu.so /tmp/keepE.so && cp tigerbeetle_amd/libtbgpu_F.so tigerbeetle_amd/libtbgpu.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_resolver.py -x -q --timeout 200 --timeout-method thread > gpurun_out/v15/pytest_F.log 2>&1 || exit 1
cp /tmp/keepE.so tigerbeetle_amd/libtbgpu.so
VARIANTS="D E F" bash tools/ab.sh cfg3 2 --host-fed-transfers 0 > gpurun_out/v15/ab.txt 2>&1
