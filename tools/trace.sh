#!/bin/bash
# rocprofv3 kernel trace + stats of one bench command (GPU box, repo root). usage: tools/trace.sh <tag> <bench args>
set -e
tag=$1; shift
out=gpurun_out/trace_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 bench.py "$@" --no-cpu-baseline > $out/bench.log 2>&1
head -25 $out/run_kernel_stats.csv | cut -d, -f1-4
