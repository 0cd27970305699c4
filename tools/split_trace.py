"""Average duration of each routed kernel (csrc/route.h) per grid size, from a rocprofv3 kernel trace.

With TBG_RT_SPLIT=1 the apply runs as three launches (home replies, side adds, record appends), each
with its own grid size, so this attributes the apply's time by role. Grids seen fewer than 20 times
(warm-up, account windows) are left out.

    python tools/split_trace.py gpurun_out/r6/trace_g8split/run_kernel_trace.csv
"""
import collections
import csv
import sys


def main(path):
    by = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if not (name.startswith("void k_rt_") or name.startswith("k_rt_")):
                continue
            key = (name.split("(")[0], int(r["Grid_Size_X"]))
            by[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    for (name, grid), v in sorted(by.items()):
        if len(v) >= 20:
            print(f"{name:28s} grid {grid:8d} n {len(v):4d} avg {sum(v) / len(v):7.2f} us")


if __name__ == "__main__":
    main(sys.argv[1])
