"""Per-kernel (and memory-copy) statistics from a rocprofv3 SQLite output (rocpd *.db): name,
calls, total / average ms, sorted by total.   python scripts/rocpd_stats.py <dir or .db> [top]"""
import glob, os, sqlite3, sys

p = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
dbs = [p] if p.endswith(".db") else glob.glob(os.path.join(p, "**", "*.db"), recursive=True)
con = sqlite3.connect(dbs[0])
cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
name = "name" if "name" in cols else "kernel_name"
rows = con.execute("select %s, count(*), sum(end - start) / 1e6, avg(end - start) / 1e6 from kernels group by %s "
                   "order by 3 desc limit %d" % (name, name, top)).fetchall()
print("%-60s %7s %10s %10s" % ("kernel", "calls", "total_ms", "avg_ms"))
for n, c, t, a in rows:
    print("%-60s %7d %10.3f %10.4f" % (n[:60], c, t, a))
try:
    mc = con.execute("select count(*), sum(end - start) / 1e6, sum(size) / 1e6 from memory_copies").fetchone()
    if mc and mc[0]:
        print("memory copies: %d, %.2f ms, %.1f MB" % mc)
        for r in con.execute("select direction, count(*), sum(end - start) / 1e6, sum(size) / 1e6 from memory_copies "
                             "group by direction"):
            print("   %s: %d copies %.2f ms %.1f MB" % r)
except sqlite3.Error as e:
    print("memory copies:", e)
