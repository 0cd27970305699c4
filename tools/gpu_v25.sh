# readlane for wave-uniform broadcasts (R, current build): full suite, cfg2 A/B vs D
mkdir -p gpurun_out/v25
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v25/pytest.log 2>&1 || exit 1
VARIANTS="D R" bash tools/ab.sh cfg2 3 --host-fed-transfers 0 > gpurun_out/v25/ab_cfg2.txt 2>&1
