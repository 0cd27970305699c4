#!/bin/bash
# Pipelined walker check on one box: the full GPU suite, then cfg4's bench line and its kernel
# statistics (results in gpurun_out/r4w/).
out=gpurun_out/r4w
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_full.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $out/pytest_full.log | head -20; tail -5 $out/pytest_full.log; exit 1; }
tail -2 $out/pytest_full.log
timeout -k 10 300 python bench.py --config cfg4 > $out/bench_cfg4.json 2> $out/bench_cfg4.err || { echo "cfg4 bench failed"; tail -5 $out/bench_cfg4.err; exit 1; }
python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('cfg4',d['value'],d['results'])" $out/bench_cfg4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/cfg4 -o run -- python3 bench.py --config cfg4 --no-cpu-baseline > $out/cfg4_trace.log 2>&1 || { echo "cfg4 trace failed"; tail -5 $out/cfg4_trace.log; exit 1; }
f=$(find $out/cfg4 -name "*kernel_stats.csv" | head -1); head -8 "$f" | cut -c1-150
