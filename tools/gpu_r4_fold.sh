#!/bin/bash
# Round 4, one box: the shard tests on E (sh_close_fold's amount sum by wave shuffles, one barrier,
# instead of a 1024-entry LDS tree), then the cfg5 A/B against D (the in-tree library).
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
out=gpurun_out/r4
cp tigerbeetle_amd/libtbgpu.so /tmp/libtbgpu.keep.so
cp tigerbeetle_amd/libtbgpu_E.so tigerbeetle_amd/libtbgpu.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_shard_dist.py tests/test_gpu_shard_general.py tests/test_gpu_shard_surface.py tests/test_gpu_bench_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_shard_E.log 2>&1
rc=$?
cp /tmp/libtbgpu.keep.so tigerbeetle_amd/libtbgpu.so
tail -2 $out/pytest_shard_E.log
[ $rc -eq 0 ] || { echo "pytest failed"; grep -E "FAILED|Error" $out/pytest_shard_E.log | head -20; exit 1; }
VARIANTS="D E" bash tools/ab.sh cfg5 3 > $out/ab_cfg5_fold_shuffles.txt 2>&1 || { echo "ab failed"; tail -5 $out/ab_cfg5_fold_shuffles.txt; exit 1; }
cat $out/ab_cfg5_fold_shuffles.txt
