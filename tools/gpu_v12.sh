# chunked resolver with per-chunk LDS sort: resolver/limit parity tests, cfg3 bench + kernel trace
mkdir -p gpurun_out/v12
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_resolver.py tests/test_gpu_bind.py tests/test_gpu_geometry.py tests/test_gpu_configs.py tests/test_gpu_kat.py -x -v --timeout 200 --timeout-method thread > gpurun_out/v12/pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config cfg3 --no-cpu-baseline --host-fed-transfers 0 > gpurun_out/v12/bench_cfg3.json 2> gpurun_out/v12/bench_cfg3.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/v12/prof -o run -- python3 bench.py --config cfg3 --no-cpu-baseline --host-fed-transfers 0 > gpurun_out/v12/prof.log 2>&1
true
