# chunked per-account sums combined in LDS (S): full suite on S, then cfg3 A/B vs D (the tree's build)
mkdir -p gpurun_out/v29
export TMPDIR=/tmp
cp tigerbeetle_amd/libtbgpu.so /tmp/keep.so && cp tigerbeetle_amd/libtbgpu_S.so tigerbeetle_amd/libtbgpu.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v29/pytest.log 2>&1 || exit 1
cp /tmp/keep.so tigerbeetle_amd/libtbgpu.so
VARIANTS="D S" bash tools/ab.sh cfg3 3 --host-fed-transfers 0 > gpurun_out/v29/ab_cfg3.txt 2>&1
