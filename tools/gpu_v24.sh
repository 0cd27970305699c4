# DPP wave scans everywhere + k_final's merged prefix pass (G, current build): full suite, cfg2 and cfg1 A/B vs D
mkdir -p gpurun_out/v24
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v24/pytest.log 2>&1 || exit 1
VARIANTS="D G" bash tools/ab.sh cfg2 3 --host-fed-transfers 0 > gpurun_out/v24/ab_cfg2.txt 2>&1
VARIANTS="D G" bash tools/ab.sh cfg1 2 --host-fed-transfers 0 > gpurun_out/v24/ab_cfg1.txt 2>&1
