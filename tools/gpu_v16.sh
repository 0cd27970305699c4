# k_ct_prep staged nontemporal event loads (P) vs default (D): parity on P, cfg2 A/B
mkdir -p gpurun_out/v16
export TMPDIR=/tmp
cp tigerbeetle_amd/libtbgpu.so /tmp/keep.so && cp tigerbeetle_amd/libtbgpu_P.so tigerbeetle_amd/libtbgpu.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_window.py tests/test_gpu_parity.py tests/test_gpu_geometry.py -x -q --timeout 200 --timeout-method thread > gpurun_out/v16/pytest_P.log 2>&1 || exit 1
cp /tmp/keep.so tigerbeetle_amd/libtbgpu.so
VARIANTS="D P" bash tools/ab.sh cfg2 3 --host-fed-transfers 0 > gpurun_out/v16/ab.txt 2>&1
