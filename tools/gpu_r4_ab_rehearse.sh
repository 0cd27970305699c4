#!/bin/bash
# Round 4: A/B of the atomics-free timing variant (libtbgpu_B.so: k_ct_fused without its balance
# adds, results wrong, timing only) against the tree's library, then the general-class rehearsals.
out=gpurun_out/r4
mkdir -p $out
export TMPDIR=/tmp
cp tigerbeetle_amd/libtbgpu.so tigerbeetle_amd/libtbgpu_A.so
VARIANTS="A B" bash tools/ab.sh cfg2 2 > $out/ab_cfg2_no_atomics.txt 2>&1 || { echo "ab failed"; exit 1; }
cat $out/ab_cfg2_no_atomics.txt
timeout -k 10 300 python tools/rehearse_shards.py --stream cfg4 --shards 8 --accounts 1000000 --transfers 4000000 --window 128 --warmup 1 > $out/rehearse_general_cfg4_g8.json 2> $out/rehearse_general_cfg4_g8.err || { echo "cfg4 rehearsal failed"; tail -5 $out/rehearse_general_cfg4_g8.err; exit 1; }
cat $out/rehearse_general_cfg4_g8.json
timeout -k 10 300 python tools/rehearse_shards.py --stream cfg3 --shards 8 --accounts 1000000 --transfers 2000000 --window 32 --warmup 1 > $out/rehearse_general_cfg3_g8.json 2> $out/rehearse_general_cfg3_g8.err || { echo "cfg3 rehearsal failed"; tail -5 $out/rehearse_general_cfg3_g8.err; exit 1; }
cat $out/rehearse_general_cfg3_g8.json
