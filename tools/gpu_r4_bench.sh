#!/bin/bash
# Round-4 bench lines on one box (repo root), each step under its own limit, results in gpurun_out/r4/:
# the default line (cfg2: host-fed + synchronous-commit lines + CPU baseline), the drop-in
# configuration (--change-log), the id orders (time-based 128-bit, random), cfg1/cfg3/cfg4/cfg5.
out=gpurun_out/r4
mkdir -p $out
export TMPDIR=/tmp
run() {  # name, limit, args... (ONLY: the names to run, default all)
  local name=$1 lim=$2; shift 2
  if [ -n "$ONLY" ] && ! [[ " $ONLY " == *" $name "* ]]; then return 0; fi
  timeout -k 10 $lim python bench.py "$@" > $out/bench_$name.json 2> $out/bench_$name.err || { echo "FAIL $name rc=$?"; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[2],d['value'],r.get('avg_launch_us'),r.get('frac'),(d.get('sync_commit') or {}).get('value'))" $out/bench_$name.json $name
}
run default 400
run cfg2_changelog 300 --change-log --no-cpu-baseline --host-fed-transfers 0 --sync-commit-batches 0
run cfg2_time 300 --id-order time --no-cpu-baseline --host-fed-transfers 0 --sync-commit-batches 0
run cfg2_time_changelog 300 --id-order time --change-log --no-cpu-baseline --host-fed-transfers 0 --sync-commit-batches 0
run cfg2_random 300 --id-order random --no-cpu-baseline --host-fed-transfers 0 --sync-commit-batches 0
run cfg1 200 --config cfg1
run cfg3 300 --config cfg3
run cfg4 300 --config cfg4
run cfg5 300 --config cfg5
