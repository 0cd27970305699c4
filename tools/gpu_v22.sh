# walker: event record prefetched one event ahead (Z: first 16 B of the next event loaded ahead): parity, cfg4 A/B vs D
mkdir -p gpurun_out/v22
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_window.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_xwin.py tests/test_gpu_pulse.py tests/test_gpu_kat.py tests/test_gpu_geometry.py -x -q --timeout 200 --timeout-method thread > gpurun_out/v22/pytest.log 2>&1 || exit 1
VARIANTS="D Z" bash tools/ab.sh cfg4 3 --host-fed-transfers 0 > gpurun_out/v22/ab.txt 2>&1
