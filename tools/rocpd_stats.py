"""Per-kernel stats from a rocprofv3 SQLite output (run_results.db; this image's default format):
  python tools/rocpd_stats.py DB [NAME_SUBSTRING ...]   -> name, calls, avg us, total ms (grid x z)"""
import sqlite3
import sys


def stats(db, keys=()):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), avg(duration), sum(duration), grid_x, grid_z from kernels "
                     "group by name, grid_x, grid_z order by sum(duration) desc").fetchall()
    out = []
    for name, n, avg, tot, gx, gz in rows:
        if keys and not any(k in name for k in keys):
            continue
        out.append((name, n, avg / 1e3, tot / 1e6, gx, gz))
    return out


if __name__ == "__main__":
    for name, n, avg, tot, gx, gz in stats(sys.argv[1], sys.argv[2:]):
        print(f"{n:6d} {avg:10.1f} us {tot:9.2f} ms  grid {gx}x{gz}  {name[:90]}")
