#!/bin/bash
# Round 4, one box: the full GPU suite (in-tree: K1), then the A/B on cfg2 with random ids (K0:
# claims inside the fused pass; K1: in a pass of their own ahead of it), then the default line.
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
out=gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_full.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $out/pytest_full.log | head -20; tail -5 $out/pytest_full.log; exit 1; }
tail -2 $out/pytest_full.log
VARIANTS="K0 K1" bash tools/ab.sh cfg2 2 --id-order random > $out/ab_cfg2_random_claim_pass.txt 2>&1 || { echo "ab failed"; tail -5 $out/ab_cfg2_random_claim_pass.txt; exit 1; }
cat $out/ab_cfg2_random_claim_pass.txt
ONLY="default" bash tools/gpu_r4_bench.sh || exit 1
