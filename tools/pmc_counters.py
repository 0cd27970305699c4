"""Per-kernel averages of arbitrary rocprofv3 --pmc counters (one pass; tools/gpu.sh pmcx).

Only the dispatches with the kernel's most common grid size are averaged (full windows).
usage: python tools/pmc_counters.py gpurun_out/r6/pmcx_<name>  -> JSON on stdout
"""
import collections
import csv
import json
import os
import sys


def short(name):
    name = name.strip('"')
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0]


def main(src):
    rows = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(os.path.join(src, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            rows[short(r["Kernel_Name"])][r["Counter_Name"]].append((int(r["Grid_Size"]), float(r["Counter_Value"])))
    out = {}
    for k, cs in rows.items():
        grids = collections.Counter(g for v in cs.values() for g, _ in v)
        grid = grids.most_common(1)[0][0]
        out[k] = {"grid": grid}
        for c, v in cs.items():
            vals = [x for g, x in v if g == grid]
            out[k][c] = sum(vals) / len(vals) if vals else None
        out[k]["dispatches"] = len([1 for g, _ in next(iter(cs.values())) if g == grid])
    top = dict(sorted(out.items(), key=lambda kv: -max((x or 0) for c, x in kv[1].items() if c not in ("grid",)))[:12])
    json.dump({"source": src, "kernels": top}, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
