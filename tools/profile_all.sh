#!/bin/bash
# Round-end rocprofv3 evidence (GPU box, repo root): cfg2 kernel trace + FETCH/WRITE passes
# (tools/profile.sh), then a kernel trace of every other config's bench line. gpurun_out/prof_*/
set -e
export TMPDIR=/tmp
bash tools/profile.sh cfg2 --host-fed-transfers 0
for c in cfg1 cfg3 cfg4 cfg5; do
  mkdir -p gpurun_out/prof_$c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$c/trace -o run -- python3 bench.py --config $c --no-cpu-baseline --host-fed-transfers 0 > gpurun_out/prof_$c/bench_trace.log 2>&1
done
find gpurun_out -path "*prof_*" -name "*kernel_stats.csv"
