# cfg4 kernel trace of the current build (rocpd db; tools/rocpd_stats.py summarizes it)
mkdir -p gpurun_out/v18
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/v18/prof -o run -- python3 bench.py --config cfg4 --no-cpu-baseline --host-fed-transfers 0 > gpurun_out/v18/prof.log 2>&1
true
