#!/bin/bash
# Round 4, one box: the shard tests on the in-tree library (D: the owner verdicts folded by
# k_sh_reply's block 0 into exchange 2's trailer, no k_sh_close launch before exchange 1), the cfg5
# A/B against C (the previous commit), then the full GPU suite.
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
out=gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_shard_dist.py tests/test_gpu_shard_general.py tests/test_gpu_shard_surface.py tests/test_gpu_bench_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_shard_D.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $out/pytest_shard_D.log | head -20; tail -3 $out/pytest_shard_D.log; exit 1; }
tail -2 $out/pytest_shard_D.log
VARIANTS="C D" bash tools/ab.sh cfg5 3 > $out/ab_cfg5_close_folded.txt 2>&1 || { echo "ab failed"; tail -5 $out/ab_cfg5_close_folded.txt; exit 1; }
cat $out/ab_cfg5_close_folded.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_full.log 2>&1 || { echo "full pytest failed"; grep -E "FAILED|Error" $out/pytest_full.log | head -20; tail -3 $out/pytest_full.log; exit 1; }
tail -2 $out/pytest_full.log
