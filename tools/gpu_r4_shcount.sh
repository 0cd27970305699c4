#!/bin/bash
# Round 4, one box: the shard tests on the in-tree library (C: k_sh_decide counts each home
# segment's failures, no k_sh_count launch), then the cfg5 A/B against B (HEAD's library).
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
out=gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_shard_dist.py tests/test_gpu_shard_general.py tests/test_gpu_shard_surface.py tests/test_gpu_bench_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_shard_C.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $out/pytest_shard_C.log | head -20; tail -3 $out/pytest_shard_C.log; exit 1; }
tail -2 $out/pytest_shard_C.log
VARIANTS="B C" bash tools/ab.sh cfg5 3 > $out/ab_cfg5_no_count_launch.txt 2>&1 || { echo "ab failed"; tail -5 $out/ab_cfg5_no_count_launch.txt; exit 1; }
cat $out/ab_cfg5_no_count_launch.txt
