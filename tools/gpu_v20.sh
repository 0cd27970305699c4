# walker: event record prefetched one event ahead (X: no scratch in the walkers, current build): parity, cfg4 A/B vs D
mkdir -p gpurun_out/v20
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_window.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_xwin.py tests/test_gpu_pulse.py tests/test_gpu_kat.py tests/test_gpu_geometry.py -x -q --timeout 200 --timeout-method thread > gpurun_out/v20/pytest.log 2>&1 || exit 1
VARIANTS="D X" bash tools/ab.sh cfg4 3 --host-fed-transfers 0 > gpurun_out/v20/ab.txt 2>&1
