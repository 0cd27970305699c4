# walker: event record prefetched one event ahead (W, current build): parity, cfg4 A/B vs D
mkdir -p gpurun_out/v19
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_window.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_xwin.py tests/test_gpu_pulse.py tests/test_gpu_kat.py tests/test_gpu_geometry.py -x -q --timeout 200 --timeout-method thread > gpurun_out/v19/pytest.log 2>&1 || exit 1
VARIANTS="D W" bash tools/ab.sh cfg4 2 --host-fed-transfers 0 > gpurun_out/v19/ab.txt 2>&1
