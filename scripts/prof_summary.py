"""Summarise a rocprofv3 run (rocpd sqlite db or kernel_stats.csv) into a text table."""
import csv, glob, os, sqlite3, sys


def rows_from(path):
    dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    if dbs:
        cur = sqlite3.connect(dbs[0]).cursor()
        return [(r[0], r[1], r[2] / 1e3, r[3] / 1e3, r[4]) for r in
                cur.execute("select name,total_calls,total_duration,average,percentage from top_kernels")]
    out = []
    for f in glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6 * 1e3 / 1e3,
                        float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    return out


if __name__ == "__main__":
    rows = rows_from(sys.argv[1])
    print(f"{'kernel':<78} {'calls':>6} {'total_us':>12} {'avg_us':>10} {'pct':>6}")
    for n, c, tot, avg, pct in rows:
        print(f"{n[:78]:<78} {c:>6} {tot*1e3 if tot < 1e3 else tot:>12.1f} {avg*1e3 if avg < 10 else avg:>10.3f} {pct:>6.2f}")
