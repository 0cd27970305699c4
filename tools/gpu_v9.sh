mkdir -p gpurun_out/v9
timeout -k 10 500 python -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_resolver.py -x -v --timeout 300 --timeout-method thread > gpurun_out/v9/pytest.log 2>&1
