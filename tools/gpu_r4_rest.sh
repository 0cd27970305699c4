#!/bin/bash
# Round 4, one box: the remaining bench lines, the abort-read A/B and the general-class rehearsals.
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
ONLY="cfg2_changelog cfg2_time cfg2_time_changelog cfg2_random cfg3 cfg5" bash tools/gpu_r4_bench.sh || exit 1
bash tools/gpu_r4_ab_rehearse2.sh || exit 1
