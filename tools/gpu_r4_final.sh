#!/bin/bash
# Round 4 final build: the full GPU suite, smoke(), and the default bench line.
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
out=gpurun_out/r4
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_full.log 2>&1 || { echo "full pytest failed"; grep -E "FAILED|Error" $out/pytest_full.log | head -20; tail -3 $out/pytest_full.log; exit 1; }
tail -2 $out/pytest_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python bench.py > $out/bench_default_final.json 2> $out/bench_default_final.err || { echo "bench failed"; tail -5 $out/bench_default_final.err; exit 1; }
tail -c 400 $out/bench_default_final.json
