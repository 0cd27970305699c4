#!/bin/bash
# Round 4, cfg5 refresh after the sharded launch folds: the bench line, rocprofv3 kernel stats and
# the two PMC passes (FETCH_SIZE, WRITE_SIZE); outputs in gpurun_out/r4/ and gpurun_out/r4p/.
export TMPDIR=/tmp
ONLY=cfg5 bash tools/gpu_r4_bench.sh || exit 1
out=gpurun_out/r4p
mkdir -p $out
B="--no-cpu-baseline --host-fed-transfers 0 --sync-commit-batches 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/cfg5/trace -o run -- python3 bench.py --config cfg5 $B > $out/cfg5_trace.log 2>&1 || { echo "cfg5 trace failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/cfg5/fetch -o run -- python3 bench.py --config cfg5 $B --no-phase-timing > $out/cfg5_fetch.log 2>&1 || { echo "cfg5 fetch failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/cfg5/write -o run -- python3 bench.py --config cfg5 $B --no-phase-timing > $out/cfg5_write.log 2>&1 || { echo "cfg5 write failed"; exit 1; }
find $out/cfg5 -name "*stats.csv"
python tools/pmc_summary.py $out/cfg5 $out/pmc_cfg5.json && head -c 600 $out/pmc_cfg5.json
