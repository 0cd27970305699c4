#!/bin/bash
# Round 4, one box: the full GPU suite, the cfg4 walker A/B (O: round-3 walker, N: walker rows, one
# 32 B row per event instead of eight column loads), then the cfg1 / cfg4 / default bench lines.
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4/pytest_full.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" gpurun_out/r4/pytest_full.log | head -20; tail -5 gpurun_out/r4/pytest_full.log; exit 1; }
tail -2 gpurun_out/r4/pytest_full.log
VARIANTS="O N" bash tools/ab.sh cfg4 3 > gpurun_out/r4/ab_cfg4_walker_rows.txt 2>&1 || { echo "walker ab failed"; tail -5 gpurun_out/r4/ab_cfg4_walker_rows.txt; exit 1; }
cat gpurun_out/r4/ab_cfg4_walker_rows.txt
ONLY="cfg1 cfg4 default" bash tools/gpu_r4_bench.sh || exit 1
