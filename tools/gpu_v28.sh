# hot ranks assigned once per block (K, current build): full suite, cfg3 and cfg2 A/B vs D
mkdir -p gpurun_out/v28
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v28/pytest.log 2>&1 || exit 1
VARIANTS="D K" bash tools/ab.sh cfg3 2 --host-fed-transfers 0 > gpurun_out/v28/ab_cfg3.txt 2>&1
VARIANTS="D K" bash tools/ab.sh cfg2 2 --host-fed-transfers 0 > gpurun_out/v28/ab_cfg2.txt 2>&1
