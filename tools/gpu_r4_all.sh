#!/bin/bash
# Round 4, one box: the full GPU suite (in-tree: C1), the claim-order A/B on cfg2 with random ids
# (C0: claim after the account probes, C1: issued behind their first loads), then the rocprofv3
# evidence (tools/gpu_r4_prof.sh).
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
out=gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_full.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $out/pytest_full.log | head -20; tail -5 $out/pytest_full.log; exit 1; }
tail -2 $out/pytest_full.log
VARIANTS="C0 C1" bash tools/ab.sh cfg2 2 --id-order random > $out/ab_cfg2_random_claim_order.txt 2>&1 || { echo "claim ab failed"; tail -5 $out/ab_cfg2_random_claim_order.txt; exit 1; }
cat $out/ab_cfg2_random_claim_order.txt
bash tools/gpu_r4_prof.sh
