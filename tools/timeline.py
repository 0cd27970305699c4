"""Device timeline from a rocprofv3 csv trace directory (kernel trace + memory-copy trace): every
kernel and copy in start order with its start offset, duration and the idle gap before it, so the
per-batch cost of the synchronous path (tools/sync_probe.py) can be split into copies, kernels and
idle time. Usage: python tools/timeline.py <dir> [--last N]"""
import argparse
import csv
import glob
import os


def rows(path, kind):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if kind == "K":
                name = r.get("Kernel_Name", "?")
            else:
                name = "%s %sB" % (r.get("Direction", "copy"), r.get("Bytes", r.get("Size", "?")))
            out.append((s, e, kind, name))
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--last", type=int, default=200)
    a = p.parse_args()
    ev = []
    for path in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        ev += rows(path, "K")
    for path in glob.glob(os.path.join(a.dir, "**", "*memory_copy_trace.csv"), recursive=True):
        ev += rows(path, "C")
    ev.sort()
    ev = ev[-a.last:]
    if not ev:
        print("no events")
        return
    t0, prev = ev[0][0], ev[0][0]
    busy = 0
    for s, e, k, n in ev:
        print("%10.1f  %7.1f us  gap %7.1f  %s %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3, k, n[:70]))
        prev = max(prev, e)
        busy += e - s
    print("span %.1f us, busy %.1f us over %d ops" % ((prev - t0) / 1e3, busy / 1e3, len(ev)))


if __name__ == "__main__":
    main()
