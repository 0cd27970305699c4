#!/bin/bash
# Round 4, one box: the full GPU suite (in-tree: NR), then the cfg4 walker A/B (D0: effects deferred
# to k_final; NR: + no record or history side stored for a component walker's creates), then cfg4.
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4/pytest_full.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" gpurun_out/r4/pytest_full.log | head -20; tail -5 gpurun_out/r4/pytest_full.log; exit 1; }
tail -2 gpurun_out/r4/pytest_full.log
VARIANTS="D0 NR" bash tools/ab.sh cfg4 3 > gpurun_out/r4/ab_cfg4_walker_norec.txt 2>&1 || { echo "walker ab failed"; tail -5 gpurun_out/r4/ab_cfg4_walker_norec.txt; exit 1; }
cat gpurun_out/r4/ab_cfg4_walker_norec.txt
