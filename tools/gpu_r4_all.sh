#!/bin/bash
# Round 4 final build, one box: the full GPU suite, every bench line, cfg4's kernel statistics.
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
out=gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_full.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $out/pytest_full.log | head -20; tail -5 $out/pytest_full.log; exit 1; }
tail -2 $out/pytest_full.log
bash tools/gpu_r4_bench.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4f/cfg4 -o run -- python3 bench.py --config cfg4 --no-cpu-baseline > gpurun_out/r4f_cfg4.log 2>&1 || { echo "cfg4 trace failed"; exit 1; }
f=$(find gpurun_out/r4f/cfg4 -name "*kernel_stats.csv" | head -1); head -6 "$f" | cut -c1-150
