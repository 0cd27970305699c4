#!/bin/bash
# Round 4, one box: the full GPU suite, the bench lines other than the default one, and the
# general-class rehearsals at G = 8 (the rocprofv3 evidence: tools/gpu_r4_prof.sh).
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
out=gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_full.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $out/pytest_full.log | head -20; tail -5 $out/pytest_full.log; exit 1; }
tail -2 $out/pytest_full.log
ONLY="cfg1 cfg2_changelog cfg2_time cfg2_time_changelog cfg2_random cfg3 cfg4 cfg5" bash tools/gpu_r4_bench.sh || exit 1
for c in "cfg4 4000000 128" "cfg3 2000000 32"; do
  set -- $c
  timeout -k 10 300 python tools/rehearse_shards.py --stream $1 --shards 8 --accounts 1000000 --transfers $2 --window $3 --warmup 1 > $out/rehearse_general_$1_g8.json 2> $out/rehearse_general_$1_g8.err || { echo "$1 rehearsal failed"; tail -5 $out/rehearse_general_$1_g8.err; exit 1; }
  cat $out/rehearse_general_$1_g8.json
done
