mkdir -p gpurun_out/d
export TMPDIR=/tmp
for r in chunks off relax; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/d/t_$r -o run -- python3 bench.py --config cfg3 --transfers 2000000 --no-cpu-baseline --resolver $r > gpurun_out/d/cfg3_$r.log 2>&1
  echo "resolver=$r rc=$?"
  grep -n "SIGSEGV\|Abort\|Segmentation\|error" gpurun_out/d/cfg3_$r.log | head -5
done
