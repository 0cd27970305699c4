# Full GPU suite without -x (every failure at once), then every config's bench line; gpurun_out/suite/
mkdir -p gpurun_out/suite
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/suite/pytest.log 2>&1
rc=$?
tail -30 gpurun_out/suite/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ -n "$NO_BENCH" ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/suite/bench_default.json 2> gpurun_out/suite/bench_default.err || exit 1
for c in ${CFGS:-cfg1 cfg3 cfg4 cfg5}; do
  timeout -k 10 300 python bench.py --config $c --host-fed-transfers 0 > gpurun_out/suite/bench_$c.json 2> gpurun_out/suite/bench_$c.err || exit 1
done
cat gpurun_out/suite/bench_*.json | cut -c1-300
exit $rc
