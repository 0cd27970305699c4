mkdir -p gpurun_out/a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_shard_general.py tests/test_gpu_hostfed.py tests/test_gpu_shard_dist.py tests/test_gpu_bench_dist.py tests/test_gpu_geometry.py -x -v --timeout 300 --timeout-method thread > gpurun_out/a/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline > gpurun_out/a/bench_cfg5.json 2> gpurun_out/a/bench_cfg5.err || exit 1
