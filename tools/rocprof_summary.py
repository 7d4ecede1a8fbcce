"""Summarise a rocprofv3 --kernel-trace run (results.db or *_kernel_stats.csv) into a markdown table."""
import csv
import sqlite3
import sys
from pathlib import Path


def rows_from_db(path):
    db = sqlite3.connect(path)
    cur = db.cursor()
    out = []
    top = cur.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    for name, calls, total, avg, pct in top:
        # top_kernels is in microseconds, the per-dispatch `duration` column in nanoseconds
        d = cur.execute("select min(duration), max(duration) from kernels where name = ?", (name,)).fetchone()
        out.append((name, int(calls), float(total), float(avg), float(d[0]) / 1e3, float(d[1]) / 1e3, float(pct)))
    return out


def rows_from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3,
                        float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3, float(r["Percentage"])))
    return out


def main(src, dst):
    p = Path(src)
    rows = rows_from_db(p) if p.suffix == ".db" else rows_from_csv(p)
    lines = ["| kernel | calls | total us | avg us | min us | max us | % |", "|---|---|---|---|---|---|---|"]
    for name, calls, tot, avg, mn, mx, pct in rows:
        short = name.split("(")[0]
        lines.append(f"| `{short}` | {calls} | {tot:.1f} | {avg:.1f} | {mn:.1f} | {mx:.1f} | {pct:.1f} |")
    Path(dst).write_text("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
