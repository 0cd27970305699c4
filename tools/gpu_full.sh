# Full GPU suite, then every config's bench line (round-end evidence); results in gpurun_out/full/
mkdir -p gpurun_out/full
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/full/bench_default.json 2> gpurun_out/full/bench_default.err || exit 1
for c in cfg1 cfg3 cfg4 cfg5; do
  timeout -k 10 300 python bench.py --config $c --host-fed-transfers 0 > gpurun_out/full/bench_$c.json 2> gpurun_out/full/bench_$c.err || exit 1
done
