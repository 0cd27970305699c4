#!/bin/bash
# rocprofv3 evidence for one bench config (run on the GPU box from the repo root):
#   kernel-trace + stats, then one PMC pass per counter (FETCH_SIZE, WRITE_SIZE), each bounded.
# usage: tools/profile.sh <tag> <bench args...>
set -e
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py "$@" --no-cpu-baseline > $out/bench_trace.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 bench.py "$@" --no-cpu-baseline --no-phase-timing > $out/bench_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 bench.py "$@" --no-cpu-baseline --no-phase-timing > $out/bench_write.log 2>&1
find $out -name "*.csv" | head -20
