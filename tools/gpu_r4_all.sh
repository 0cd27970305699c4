#!/bin/bash
# Round 4, one box: the full GPU suite, then the bench lines, the cfg4 walker A/B (O: round-3
# walker, R: pipelined with records in registers, T: pipelined with records touched ahead), then
# the abort-read A/B and the general-class rehearsals.
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4/pytest_full.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" gpurun_out/r4/pytest_full.log | head -20; tail -5 gpurun_out/r4/pytest_full.log; exit 1; }
tail -2 gpurun_out/r4/pytest_full.log
VARIANTS="O R T" bash tools/ab.sh cfg4 2 > gpurun_out/r4/ab_cfg4_walker.txt 2>&1 || { echo "walker ab failed"; tail -5 gpurun_out/r4/ab_cfg4_walker.txt; exit 1; }
cat gpurun_out/r4/ab_cfg4_walker.txt
bash tools/gpu_r4_bench.sh || exit 1
bash tools/gpu_r4_ab_rehearse2.sh || exit 1
