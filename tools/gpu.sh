#!/bin/bash
# One parameterised driver for GPU-box runs (repo root, under gpurun). Each step runs under its own
# time limit and the first failure ends the script. Results go to gpurun_out/$OUT (default r5/).
#   tools/gpu.sh test [pytest -k expr]     the GPU suite (or a selection)
#   tools/gpu.sh smoke                     __graft_entry__.smoke()
#   tools/gpu.sh bench NAME [bench args]   one bench line -> bench_NAME.json (+ a one-line summary)
#   tools/gpu.sh prof NAME [bench args]    rocprofv3 kernel trace + stats of one bench line, then one
#                                          PMC pass per counter (FETCH_SIZE, WRITE_SIZE), summarised by
#                                          tools/pmc_summary.py into pmc_NAME.json
#   tools/gpu.sh pmcx NAME "CTRS" [bench args]  one PMC pass with the given counters (tools/pmc_counters.py)
#   tools/gpu.sh profpy NAME script [args] the same passes over any script (e.g. tools/rehearse_shards.py)
#   tools/gpu.sh pmcpy NAME "CTRS" script [args]  one PMC pass with the given counters over any script
#   tools/gpu.sh rehearse NAME [args]      tools/rehearse_shards.py -> rehearse_NAME.json
#   tools/gpu.sh py NAME script [args]     any probe script (tools/*.py) -> NAME.json
#   tools/gpu.sh trace NAME script [args]  rocprofv3 kernel trace + stats of a script -> trace_NAME/
#   tools/gpu.sh timeline NAME script [args]  kernel + memory-copy trace, the last ops in start order
#                                          (tools/timeline.py) -> timeline_NAME/
# Several commands chain with "+": tools/gpu.sh test + bench default + prof cfg2 --config cfg2
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${OUT:-r5}
mkdir -p $out
B="--no-cpu-baseline --host-fed-transfers 0 --sync-commit-batches 0"

summary() {  # bench json -> value, roofline kernel avg launch, frac, sync line
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(sys.argv[2],d['value'],r.get('avg_launch_us'),r.get('frac'),(d.get('sync_commit') or {}).get('value'))" "$1" "$2"
}

pmc_passes() {  # NAME cmd...: kernel trace + stats, then one PMC pass per counter -> pmc_NAME.json
  local name=$1; shift
  local d=$out/prof_$name
  mkdir -p $d
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d/trace -o run -- "$@" > $d/trace.log 2>&1 || { echo "trace $name failed"; tail -5 $d/trace.log; return 1; }
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/fetch -o run -- "$@" > $d/fetch.log 2>&1 || { echo "fetch $name failed"; return 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/write -o run -- "$@" > $d/write.log 2>&1 || { echo "write $name failed"; return 1; }
  python tools/pmc_summary.py $d $out/pmc_$name.json && head -c 600 $out/pmc_$name.json; echo
}

step() {
  local cmd=$1; shift
  case $cmd in
    test)
      local sel=()
      [ -n "$1" ] && sel=(-k "$1")
      timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${sel[@]}" \
        > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $out/pytest.log | head -20; tail -3 $out/pytest.log; return 1; }
      tail -1 $out/pytest.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $out/smoke.log; return 1; }
      tail -1 $out/smoke.log ;;
    bench)
      local name=$1; shift
      timeout -k 10 400 python bench.py "$@" > $out/bench_$name.json 2> $out/bench_$name.err || { echo "bench $name failed"; tail -5 $out/bench_$name.err; return 1; }
      summary $out/bench_$name.json $name ;;
    prof)
      local name=$1; shift
      pmc_passes $name python3 bench.py $B "$@" --no-phase-timing || return 1 ;;
    pmcx)  # NAME "COUNTERS" [bench args]: one PMC pass with the given counters over a bench line
      local name=$1 ctrs=$2; shift 2
      local d=$out/pmcx_$name
      mkdir -p $d
      timeout -s KILL 300 rocprofv3 --pmc $ctrs --output-format csv -d $d -o run -- python3 bench.py $B "$@" --no-phase-timing > $d/run.log 2>&1 || { echo "pmcx $name failed"; tail -3 $d/run.log; return 1; }
      python tools/pmc_counters.py $d > $out/pmcx_$name.json && head -c 800 $out/pmcx_$name.json; echo ;;
    pmcpy)  # NAME "COUNTERS" script [args]: one PMC pass with the given counters over any script
      local name=$1 ctrs=$2; shift 2
      local d=$out/pmcx_$name
      mkdir -p $d
      timeout -s KILL 300 rocprofv3 --pmc $ctrs --output-format csv -d $d -o run -- python3 -u "$@" > $d/run.log 2>&1 || { echo "pmcpy $name failed"; tail -3 $d/run.log; return 1; }
      python tools/pmc_counters.py $d > $out/pmcx_$name.json && head -c 1500 $out/pmcx_$name.json; echo ;;
    profpy)
      local name=$1; shift
      pmc_passes $name python3 -u "$@" || return 1 ;;
    rehearse)
      local name=$1; shift
      timeout -k 10 600 python -u tools/rehearse_shards.py "$@" > $out/rehearse_$name.json 2> $out/rehearse_$name.err || { echo "rehearse $name failed"; tail -5 $out/rehearse_$name.err; return 1; }
      tail -c 1500 $out/rehearse_$name.json ;;
    trace)
      local name=$1; shift
      local d=$out/trace_$name
      mkdir -p $d
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 -u "$@" > $d/run.log 2>&1 || { echo "trace $name failed"; tail -5 $d/run.log; return 1; }
      python tools/kstats.py $d/run_kernel_stats.csv ;;
    timeline)
      local name=$1; shift
      local d=$out/timeline_$name
      mkdir -p $d
      timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $d -o run -- python3 -u "$@" > $d/run.log 2>&1 || { echo "timeline $name failed"; tail -5 $d/run.log; return 1; }
      python tools/timeline.py $d --last ${LAST:-120} > $d/timeline.txt && tail -40 $d/timeline.txt ;;
    py)
      local name=$1; shift
      timeout -k 10 600 python -u "$@" > $out/$name.json 2> $out/$name.err || { echo "$name failed"; tail -5 $out/$name.err; return 1; }
      tail -c 1500 $out/$name.json ;;
    *) echo "unknown step $cmd"; return 1 ;;
  esac
}

args=()
for a in "$@" +; do
  if [ "$a" = "+" ]; then
    [ ${#args[@]} -gt 0 ] && { step "${args[@]}" || exit 1; }
    args=()
  else
    args+=("$a")
  fi
done
