# cfg2 (default bench) kernel trace of the final build: stats csv (or the rocpd db)
mkdir -p gpurun_out/v27
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v27/prof -o run -- python3 bench.py > gpurun_out/v27/bench.json 2> gpurun_out/v27/prof.err
true
