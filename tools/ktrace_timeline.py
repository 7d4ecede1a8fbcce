"""Timeline of a rocprofv3 kernel trace: one line per dispatch (start / end relative to the first dispatch of
the chosen step, queue id, kernel, grid), for steps [first, first + n) of a small-batch trace.  A step starts
at every k_resize_cascade dispatch of queue 0's kind, i.e. every `handles`-th cascade.
usage: python tools/ktrace_timeline.py TRACE_DIR [--handles H] [--first 20] [--n 2]"""
import argparse
import csv
import glob


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--handles", type=int, default=1)
    ap.add_argument("--first", type=int, default=20)
    ap.add_argument("--n", type=int, default=2)
    a = ap.parse_args()
    rows = []
    for f in glob.glob(f"{a.trace}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("orbfe::", "")
            grid = f'{r.get("Grid_Size_X", r.get("Grid_Size", "?"))}x{r.get("Grid_Size_Y", "")}'
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", r.get("Stream_Id", "?")),
                         grid))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[2] in ("k_resize_cascade", "k_resize_rows")]
    starts = starts[::a.handles]
    i0 = starts[a.first]
    i1 = starts[a.first + a.n] if a.first + a.n < len(starts) else len(rows)
    t0 = rows[i0][0]
    for s, e, n, q, g in rows[i0:i1]:
        print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q{q:>3} {n:22s} {g}")


if __name__ == "__main__":
    main()
