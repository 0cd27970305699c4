# Tests named in $TESTS, then A/B timing per config in $CFGS over $VARIANTS (results in gpurun_out/g/)
mkdir -p gpurun_out/g
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest ${TESTS} -x -q --timeout 120 --timeout-method thread > gpurun_out/g/t.log 2>&1
rc=$?
tail -3 gpurun_out/g/t.log
[ $rc -ne 0 ] && exit $rc
for c in ${CFGS}; do
  VARIANTS="${VARIANTS}" bash tools/ab.sh $c ${ROUNDS:-2} > gpurun_out/g/ab_$c.txt 2>&1 || exit 1
  cut -c1-200 gpurun_out/g/ab_$c.txt
done
