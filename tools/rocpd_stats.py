"""Per-kernel call count / average duration from a rocprofv3 results.db (when the csv step crashed)."""
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in con.execute("pragma table_info(rocpd_kernel_dispatch)")]
ks = [r[1] for r in con.execute("pragma table_info(rocpd_info_kernel_symbol)")]
name_col = "kernel_name" if "kernel_name" in ks else ("display_name" if "display_name" in ks else ks[1])
q = f"""select s.{name_col}, count(*), avg(d.end - d.start), sum(d.end - d.start)
        from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
        group by s.{name_col} order by sum(d.end - d.start) desc"""
rows = list(con.execute(q))
tot = sum(r[3] for r in rows)
print("Name,Calls,AverageNs,Percentage")
for n, c, a, s in rows:
    print(f'"{n}",{c},{a:.1f},{100.0 * s / tot:.2f}')
