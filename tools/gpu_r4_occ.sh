#!/bin/bash
# Round 4, one box: fewer resident waves for the random-access kernels. cfg2: k_ct_fused held to
# 5 / 4 / 3 blocks (waves per SIMD) per CU by dynamic LDS (F5 / F4 / F3) against B (HEAD: 6);
# cfg5: k_sh_owned_ct held to one 1024-thread block per CU (O4) against B (two).
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
out=gpurun_out/r4
VARIANTS="B F5 F4 F3" bash tools/ab.sh cfg2 2 > $out/ab_cfg2_fused_fewer_waves.txt 2>&1 || { echo "ab cfg2 failed"; tail -5 $out/ab_cfg2_fused_fewer_waves.txt; exit 1; }
cat $out/ab_cfg2_fused_fewer_waves.txt
VARIANTS="B O4" bash tools/ab.sh cfg5 2 > $out/ab_cfg5_owned_fewer_waves.txt 2>&1 || { echo "ab cfg5 failed"; tail -5 $out/ab_cfg5_owned_fewer_waves.txt; exit 1; }
cat $out/ab_cfg5_owned_fewer_waves.txt
