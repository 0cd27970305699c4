# limit-path tests on the current build, then a cfg3 A/B of library variants B C D
mkdir -p gpurun_out/v13
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_resolver.py tests/test_gpu_bind.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/v13/pytest.log 2>&1 || exit 1
VARIANTS="B C D" bash tools/ab.sh cfg3 2 --host-fed-transfers 0 > gpurun_out/v13/ab.txt 2>&1
