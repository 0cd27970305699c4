#!/bin/bash
# Round 4, one box: the full GPU suite (in-tree: Z), then the cfg4 A/B (Y: k_ct_prep claims before
# the lookups; Z: after them).
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
out=gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_full.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $out/pytest_full.log | head -20; tail -5 $out/pytest_full.log; exit 1; }
tail -2 $out/pytest_full.log
VARIANTS="Y Z" bash tools/ab.sh cfg4 3 > $out/ab_cfg4_prep_claims_last.txt 2>&1 || { echo "ab failed"; tail -5 $out/ab_cfg4_prep_claims_last.txt; exit 1; }
cat $out/ab_cfg4_prep_claims_last.txt
