#!/bin/bash
# All bench lines + kernel stats for one round (GPU box, repo root): results in gpurun_out/r2/.
set -e
out=gpurun_out/r2
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $out/bench_default.json 2> $out/bench_default.err
for c in cfg1 cfg3 cfg4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --host-fed-transfers 0 > $out/bench_$c.json 2> $out/bench_$c.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_cfg2 -o run -- python3 bench.py --no-cpu-baseline --host-fed-transfers 0 > $out/prof_cfg2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_cfg4 -o run -- python3 bench.py --config cfg4 --no-cpu-baseline --host-fed-transfers 0 > $out/prof_cfg4.log 2>&1
find $out -name "*stats.csv"
