# Full GPU suite, then the default (cfg2) and cfg4 bench lines; results in gpurun_out/v11/
mkdir -p gpurun_out/v11
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v11/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/v11/bench_default.json 2> gpurun_out/v11/bench_default.err || exit 1
timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline --host-fed-transfers 0 > gpurun_out/v11/bench_cfg4.json 2> gpurun_out/v11/bench_cfg4.err || exit 1
