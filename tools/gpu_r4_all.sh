#!/bin/bash
# Round 4, one box: the full GPU suite (in-tree: S1), then the cfg2 A/B (S0: k_fu_final with its
# record temp in scratch memory; S1: in registers; W7 / W8: S1 with k_ct_fused held to 7 / 8 waves
# per SIMD, 20 / 60 B of scratch).
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
out=gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_full.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $out/pytest_full.log | head -20; tail -5 $out/pytest_full.log; exit 1; }
tail -2 $out/pytest_full.log
VARIANTS="S0 S1 W7 W8" bash tools/ab.sh cfg2 2 > $out/ab_cfg2_fu_final_scratch.txt 2>&1 || { echo "ab failed"; tail -5 $out/ab_cfg2_fu_final_scratch.txt; exit 1; }
cat $out/ab_cfg2_fu_final_scratch.txt
