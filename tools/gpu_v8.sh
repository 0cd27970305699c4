mkdir -p gpurun_out/v8
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v8/prof_cfg3 -o run -- python3 bench.py --config cfg3 --no-cpu-baseline --host-fed-transfers 0 > gpurun_out/v8/prof_cfg3.log 2>&1
echo rc=$? >> gpurun_out/v8/prof_cfg3.log
