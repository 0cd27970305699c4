# Round-end evidence: smoke, full GPU suite, every config's bench line; results in gpurun_out/full/
mkdir -p gpurun_out/full
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full/smoke.log 2>&1 || exit 1
bash tools/gpu_full.sh
