# chunked resolver with deferred result stores (F: next-chunk fetch in the first walk phase, current build): limit-path parity, cfg3 A/B vs D
mkdir -p gpurun_out/v23
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_resolver.py tests/test_gpu_bind.py tests/test_gpu_configs.py tests/test_gpu_geometry.py -x -q --timeout 200 --timeout-method thread > gpurun_out/v23/pytest.log 2>&1 || exit 1
VARIANTS="D F" bash tools/ab.sh cfg3 3 --host-fed-transfers 0 > gpurun_out/v23/ab.txt 2>&1
