"""Idle gaps between consecutive kernel dispatches (rocprofv3 results.db): total, and the largest by
the kernel that follows the gap."""
import collections
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
ks = [r[1] for r in con.execute("pragma table_info(rocpd_info_kernel_symbol)")]
name_col = "kernel_name" if "kernel_name" in ks else ks[1]
rows = list(con.execute(f"""select d.start, d.end, s.{name_col} from rocpd_kernel_dispatch d
                            join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start"""))
gaps = collections.defaultdict(list)
busy = 0
for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
    g = s1 - e0
    if 0 < g < 2_000_000:
        gaps[(n0[:40], n1[:40])].append(g)
for k, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[:25]:
    print(f"{sum(v) / 1000:10.1f} us  n={len(v):5d}  avg={sum(v) / len(v) / 1000:7.2f} us  {k[0]} -> {k[1]}")
