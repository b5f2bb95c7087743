"""Kernel statistics (the rocprofv3 --stats CSV columns) from a rocprofv3 rocpd database
(rocprofv3's default output on this image): per kernel name, calls, total / average / min /
max duration in ns, percentage.  usage: python profiles/rocpd_stats.py <run_results.db> [out.csv]"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("SELECT name, start, end FROM kernels").fetchall()
    acc = {}
    for name, s, e in rows:
        a = acc.setdefault(name, [])
        a.append(e - s)
    total = sum(sum(v) for v in acc.values()) or 1
    out = []
    for name, d in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        out.append({"Name": name, "Calls": len(d), "TotalDurationNs": sum(d), "AverageNs": sum(d) / len(d),
                    "Percentage": 100.0 * sum(d) / total, "MinNs": min(d), "MaxNs": max(d)})
    return out


if __name__ == "__main__":
    res = stats(sys.argv[1])
    w = csv.DictWriter(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout, fieldnames=list(res[0]))
    w.writeheader()
    for r in res:
        w.writerow(r)
