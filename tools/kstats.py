"""Prints a rocprofv3 kernel_stats.csv (name, calls, average us, share): python tools/kstats.py <csv>"""
import csv
import sys

for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    print(path)
    for r in rows[:30]:
        print("  %-60s %7s %10.1f us %6s %%" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1000.0,
                                                r["Percentage"][:6]))
