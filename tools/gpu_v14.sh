# cfg3 kernel trace of the current build (rocpd db; tools/rocpd_stats.py summarizes it)
mkdir -p gpurun_out/v14
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/v14/prof -o run -- python3 bench.py --config cfg3 --no-cpu-baseline --host-fed-transfers 0 > gpurun_out/v14/prof.log 2>&1
true
