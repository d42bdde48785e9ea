"""Per-kernel statistics from a rocprofv3 SQLite database (rocpd schema, ROCm 7.2 default output):
calls, average / total device time and share.  Usage: python scripts/rocpd_stats.py DB [TOP] [--csv OUT]"""
import collections
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    names = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    agg = collections.defaultdict(lambda: [0, 0.0, None])
    for kid, s, e, gx, gy, gz, wx in c.execute(
            "select kernel_id, start, end, grid_size_x, grid_size_y, grid_size_z, workgroup_size_x "
            "from rocpd_kernel_dispatch"):
        a = agg[names.get(kid, str(kid))]
        a[0] += 1
        a[1] += (e - s)
        a[2] = (gx // max(1, wx), gy, gz)
    tot = sum(v[1] for v in agg.values())
    rows = sorted(((k, v[0], v[1] / v[0] / 1e3, v[1] / 1e3, 100.0 * v[1] / tot, v[2]) for k, v in agg.items()),
                  key=lambda r: -r[3])
    return rows, tot


if __name__ == "__main__":
    db = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 20
    rows, tot = stats(db)
    print("total kernel time %.1f ms" % (tot / 1e6))
    for name, calls, avg, total, pct, grid in rows[:top]:
        print("%6d  %9.1f us  %10.1f us  %5.1f%%  grid %-16s %s" % (calls, avg, total, pct, grid, name[:110]))
    if "--csv" in sys.argv:
        with open(sys.argv[sys.argv.index("--csv") + 1], "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "AverageUs", "TotalUs", "Percent", "Grid"])
            for r in rows:
                w.writerow([r[0], r[1], round(r[2], 2), round(r[3], 1), round(r[4], 2), r[5]])
