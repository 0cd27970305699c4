#!/bin/bash
# Round 4 step 2: fused / sharded-general GPU tests, A/B of the abort-read change, general rehearsals.
out=gpurun_out/r4
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_shard_general.py tests/test_gpu_shard_surface.py tests/test_gpu_restore.py -x -q --timeout 300 --timeout-method thread > $out/pytest_step2.log 2>&1 || { echo "pytest failed"; tail -20 $out/pytest_step2.log; exit 1; }
tail -2 $out/pytest_step2.log
VARIANTS="A B" bash tools/ab.sh cfg2 3 > $out/ab_cfg2_abort_read.txt 2>&1 || { echo "ab failed"; exit 1; }
cat $out/ab_cfg2_abort_read.txt
timeout -k 10 300 python tools/rehearse_shards.py --stream cfg4 --shards 8 --accounts 1000000 --transfers 4000000 --window 128 --warmup 1 > $out/rehearse_general_cfg4_g8.json 2> $out/rehearse_general_cfg4_g8.err || { echo "cfg4 rehearsal failed"; tail -5 $out/rehearse_general_cfg4_g8.err; exit 1; }
cat $out/rehearse_general_cfg4_g8.json
timeout -k 10 300 python tools/rehearse_shards.py --stream cfg3 --shards 8 --accounts 1000000 --transfers 2000000 --window 32 --warmup 1 > $out/rehearse_general_cfg3_g8.json 2> $out/rehearse_general_cfg3_g8.err || { echo "cfg3 rehearsal failed"; tail -5 $out/rehearse_general_cfg3_g8.err; exit 1; }
cat $out/rehearse_general_cfg3_g8.json
