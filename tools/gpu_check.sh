# Targeted GPU check: the tests named in $TESTS, then an A/B of $CFG (results in gpurun_out/a/)
mkdir -p gpurun_out/a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS} -x -v --timeout 300 --timeout-method thread > gpurun_out/a/pytest.log 2>&1 || exit 1
if [ -n "$CFG" ]; then VARIANTS="${VARIANTS:-A B}" bash tools/ab.sh $CFG ${ROUNDS:-2} > gpurun_out/a/ab.txt 2>&1 || exit 1; fi
