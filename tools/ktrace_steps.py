"""Per-step view of a rocprofv3 kernel trace of tools/small_trace.py: kernels grouped into steps (a step
starts at each k_resize_cascade, or at every 7th k_resize_rows dispatch, i.e. level 1), per step the span from the first
kernel's start to the last one's end, the summed kernel time and the idle gaps; per kernel the median
duration.  usage: python tools/ktrace_steps.py TRACE_DIR [skip_steps]"""
import collections
import csv
import glob
import statistics
import sys


def main():
    d = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    rows = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("orbfe::", "")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    steps, cur, nres = [], [], 0
    for s, e, n in rows:
        if n == "k_resize_rows" or n == "k_resize_cascade":
            if (n == "k_resize_cascade" or nres % 7 == 0) and cur:
                steps.append(cur)
                cur = []
            nres += n == "k_resize_rows"
        cur.append((s, e, n))
    if cur:
        steps.append(cur)
    steps = steps[skip:]
    span, busy, gaps = [], [], []
    per = collections.defaultdict(list)
    for st in steps:
        span.append((st[-1][1] - st[0][0]) / 1e3)
        busy.append(sum(e - s for s, e, _ in st) / 1e3)
        g = 0
        for (s0, e0, _), (s1, e1, _) in zip(st, st[1:]):
            g += max(0, s1 - e0)
        gaps.append(g / 1e3)
        cnt = collections.Counter()
        for s, e, n in st:
            per[(n, cnt[n])].append((e - s) / 1e3)
            cnt[n] += 1
    print(f"steps {len(steps)}: span p50 {statistics.median(span):.1f} us, kernel time p50 "
          f"{statistics.median(busy):.1f} us, idle gaps p50 {statistics.median(gaps):.1f} us, "
          f"kernels per step {len(steps[0]) if steps else 0}")
    for (n, i), v in sorted(per.items(), key=lambda kv: -statistics.median(kv[1])):
        print(f"  {n:20s} #{i}  median {statistics.median(v):8.1f} us")


if __name__ == "__main__":
    main()
