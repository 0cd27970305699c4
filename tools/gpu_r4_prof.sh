#!/bin/bash
# Round-4 rocprofv3 evidence: kernel-trace + stats of the default bench line (cfg2) and of cfg4 and
# cfg5, then one PMC pass per counter (FETCH_SIZE, WRITE_SIZE) over cfg2; summaries to gpurun_out/r4p/.
out=gpurun_out/r4p
mkdir -p $out
export TMPDIR=/tmp
B="--no-cpu-baseline --host-fed-transfers 0 --sync-commit-batches 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/cfg2/trace -o run -- python3 bench.py $B > $out/cfg2_trace.log 2>&1 || { echo "cfg2 trace failed"; tail -5 $out/cfg2_trace.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/cfg2/fetch -o run -- python3 bench.py $B --no-phase-timing > $out/cfg2_fetch.log 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/cfg2/write -o run -- python3 bench.py $B --no-phase-timing > $out/cfg2_write.log 2>&1 || { echo "write pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/cfg4/trace -o run -- python3 bench.py --config cfg4 $B > $out/cfg4_trace.log 2>&1 || { echo "cfg4 trace failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/cfg5/trace -o run -- python3 bench.py --config cfg5 $B > $out/cfg5_trace.log 2>&1 || { echo "cfg5 trace failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/cfg5/fetch -o run -- python3 bench.py --config cfg5 $B --no-phase-timing > $out/cfg5_fetch.log 2>&1 || { echo "cfg5 fetch failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/cfg5/write -o run -- python3 bench.py --config cfg5 $B --no-phase-timing > $out/cfg5_write.log 2>&1 || { echo "cfg5 write failed"; exit 1; }
find $out -name "*stats.csv" -o -name "*counter_collection.csv" | head -20
python tools/pmc_summary.py $out/cfg2 $out/pmc_cfg2.json && head -c 1500 $out/pmc_cfg2.json
python tools/pmc_summary.py $out/cfg5 $out/pmc_cfg5.json && head -c 600 $out/pmc_cfg5.json
