# DPP u64 min-scan in the pulse_next replays (M, current build): full suite, cfg4 A/B vs D
mkdir -p gpurun_out/v26
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v26/pytest.log 2>&1 || exit 1
VARIANTS="D M" bash tools/ab.sh cfg4 3 --host-fed-transfers 0 > gpurun_out/v26/ab_cfg4.txt 2>&1
