#!/bin/bash
# A/B of the abort-read change (A: round-3 block-barrier read, B: per-wave read in the vote), then the
# general-class rehearsals at G = 8.
out=gpurun_out/r4
export TMPDIR=/tmp
VARIANTS="A B" bash tools/ab.sh cfg2 3 > $out/ab_cfg2_abort_read.txt 2>&1 || { echo "ab failed"; exit 1; }
cat $out/ab_cfg2_abort_read.txt
for c in "cfg4 4000000 128" "cfg3 2000000 32"; do
  set -- $c
  timeout -k 10 300 python tools/rehearse_shards.py --stream $1 --shards 8 --accounts 1000000 --transfers $2 --window $3 --warmup 1 > $out/rehearse_general_$1_g8.json 2> $out/rehearse_general_$1_g8.err || { echo "$1 rehearsal failed"; tail -5 $out/rehearse_general_$1_g8.err; exit 1; }
  cat $out/rehearse_general_$1_g8.json
done
