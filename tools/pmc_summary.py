"""Summarize rocprofv3 output of tools/profile.sh into profiles/<round>/pmc_<tag>.json.

Per kernel: launches, average duration (kernel-trace --stats), and per-launch FETCH_SIZE / WRITE_SIZE
from the separate --pmc passes (rocprofv3 reports them in KiB; bytes here). Only the dispatches with
the kernel's most common grid size are averaged (full commit windows; the warm-up tail and the setup
windows have other sizes). bench.py reads `traffic` for its roofline kernel from this file.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts 64 B per TCC_EA read request and
reports half the bytes of wide 16 B/lane streaming reads; other access widths are uncalibrated. The
summary keeps the raw counter bytes and an x2-corrected fetch alongside (bounds, not one number).

usage: python tools/pmc_summary.py gpurun_out/prof_cfg2 profiles/r1/pmc_cfg2.json
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


def load_counter(path, counter):
    rows = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                rows[short(r["Kernel_Name"])].append((int(r["Grid_Size"]), float(r["Counter_Value"])))
    out = {}
    for k, v in rows.items():
        grid = collections.Counter(g for g, _ in v).most_common(1)[0][0]
        vals = [x for g, x in v if g == grid]
        out[k] = (grid, len(vals), 1024.0 * sum(vals) / len(vals))
    return out


def main(src, dst):
    stats = {}
    with open(os.path.join(src, "trace", "run_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                       "percent": float(r["Percentage"])}
    fetch = load_counter(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = load_counter(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    kernels = {}
    for k, st in sorted(stats.items(), key=lambda kv: -kv[1]["percent"]):
        if k not in fetch or k not in write:
            continue
        grid, n, fb = fetch[k]
        _, _, wb = write[k]
        kernels[k] = dict(st, grid=grid, pmc_dispatches=n, fetch_bytes=round(fb), write_bytes=round(wb),
                          traffic_bytes=round(fb + wb), traffic_fetch_x2_bytes=round(2 * fb + wb))
    with open(dst, "w") as f:
        json.dump({"source": src, "kernels": kernels}, f, indent=1)
    for k, v in list(kernels.items())[:8]:
        print(f"{k:28s} {v['calls']:5d} calls {v['avg_ns'] / 1000:9.1f} us  fetch {v['fetch_bytes'] / 1e6:8.1f} MB"
              f"  write {v['write_bytes'] / 1e6:8.1f} MB  (grid {v['grid']})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
