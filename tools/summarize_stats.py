"""Summarise rocprofv3 kernel stats: top kernels by total time.

Accepts either the `--stats` kernel CSV (`*_kernel_stats.csv`) or the rocpd SQLite database
(`*_results.db`) that rocprofv3 writes by default.

    python tools/summarize_stats.py FILE [TOP_N]
"""
import csv
import sqlite3
import sys


def rows_from_csv(path):
    out = []
    for r in csv.DictReader(open(path)):
        out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"])))
    return out


def rows_from_db(path):
    c = sqlite3.connect(path)
    q = ("select name, count(*), sum(end - start), avg(end - start) from kernels "
         "group by name")
    return [(n, int(k), float(t), float(a)) for n, k, t, a in c.execute(q)]


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rows = rows_from_db(path) if path.endswith(".db") else rows_from_csv(path)
    tot = sum(r[2] for r in rows)
    print(f"{'total ms':>9} {'%':>6} {'calls':>7} {'avg us':>9}  kernel")
    for name, calls, total, avg in sorted(rows, key=lambda r: -r[2])[:n]:
        print(f"{total / 1e6:9.2f} {100 * total / tot:6.2f} {calls:>7} {avg / 1e3:9.2f}  {name[:100]}")
    print(f"sum of kernel time: {tot / 1e6:.1f} ms over {sum(r[1] for r in rows)} launches")


if __name__ == "__main__":
    main()
