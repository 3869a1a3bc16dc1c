"""Summarise a rocprofv3 SQLite (rocpd) database: per-kernel dispatch stats."""
import sqlite3, sys, json
db = sys.argv[1]
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(rocpd_kernel_dispatch)")]
q = """select s.kernel_name as name, count(*) as calls, sum(d.end - d.start) as total_ns,
              avg(d.end - d.start) as avg_ns, min(d.end - d.start) as min_ns, max(d.end - d.start) as max_ns
       from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
       group by s.kernel_name order by total_ns desc"""
rows = c.execute(q).fetchall()
tot = sum(r[2] for r in rows) or 1
print(f"{'kernel':<70} {'calls':>6} {'total_ms':>10} {'avg_us':>10} {'pct':>6}")
for name, calls, total, avg, mn, mx in rows:
    print(f"{name[:70]:<70} {calls:>6} {total/1e6:>10.3f} {avg/1e3:>10.1f} {100*total/tot:>6.1f}")
