"""Sum rocprofv3 --pmc counters per kernel (all launches of all template variants merged by base
template arguments) (development aid).  usage: python tools/pmc_agg.py DIR [DIR ...]"""
import collections
import csv
import glob
import re
import sys

for d in sys.argv[1:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(set)
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_\w+)(<(\d+))?", r["Kernel_Name"])
            if not m:
                continue
            key = m.group(1) + (f"<{m.group(3)}>" if m.group(3) else "")
            acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
            n[key].add(r.get("Dispatch_Id", r.get("Dispatch_ID", "")))
    print(d)
    for k, cs in acc.items():
        print(f"  {k:18s} dispatches={len(n[k]):4d} " + " ".join(f"{c}={v / 1e6:.2f}M" for c, v in sorted(cs.items())))
