# cfg3 with RC_PROF builds of the library (per-phase cycles of k_rc_run into the debug counters):
# PROFS="P2 P3" bash tools/rc_prof.sh  (libtbgpu_<P>.so; the tree's library is restored on exit)
cp tigerbeetle_amd/libtbgpu.so /tmp/libtbgpu.keep.so
trap 'cp /tmp/libtbgpu.keep.so tigerbeetle_amd/libtbgpu.so' EXIT
mkdir -p gpurun_out/p
for v in ${PROFS:-P}; do
  cp tigerbeetle_amd/libtbgpu_$v.so tigerbeetle_amd/libtbgpu.so
  TBG_DEBUG=1 timeout -k 10 300 python bench.py --config cfg3 --no-cpu-baseline --host-fed-transfers 0 > gpurun_out/p/cfg3_$v.json 2> gpurun_out/p/cfg3_$v.err || exit 1
  echo "$v $(grep 'resolver counters' gpurun_out/p/cfg3_$v.err)"
done
