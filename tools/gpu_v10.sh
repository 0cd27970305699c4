mkdir -p gpurun_out/v10
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/v10/pmc -o run -- python3 tools/cfg3_probe.py 3 32 > gpurun_out/v10/pmc.log 2>&1
echo rc=$? >> gpurun_out/v10/pmc.log
