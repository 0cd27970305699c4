#!/bin/bash
# cfg4 kernel trace (the in-tree library): per-kernel start/end of the component walkers.
out=gpurun_out/r4t
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/cfg4 -o run -- python3 bench.py --config cfg4 --no-cpu-baseline --no-phase-timing > $out/cfg4_trace.log 2>&1 || { echo "trace failed"; tail -5 $out/cfg4_trace.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r4t/cfg4/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ks = [r for r in rows if "k_cc_walk" in r["Kernel_Name"] or "k_cc_segs" in r["Kernel_Name"] or "k_walk<" in r["Kernel_Name"]]
for r in ks[-12:]:
    print(r["Kernel_Name"][:40], r["Start_Timestamp"], r["End_Timestamp"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
PY
f=$(find $out/cfg4 -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -c1-160
