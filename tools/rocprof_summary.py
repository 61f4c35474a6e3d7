"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd SQLite output) into a kernel-stats CSV:
name, calls, total_us, avg_us, min_us, max_us, percent.  Usage: rocprof_summary.py <results.db> <out.csv>"""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["name", "calls", "total_us", "avg_us", "min_us", "max_us", "percent"])
        for name, n, tot, avg, mn, mx in rows:
            w.writerow([name, n, round(tot / 1e3, 3), round(avg / 1e3, 3), round(mn / 1e3, 3), round(mx / 1e3, 3),
                        round(100.0 * tot / total, 3)])
    for r in rows[:8]:
        print("%-70s %6d avg %10.2f us" % (r[0][:70], r[1], r[3] / 1e3))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
