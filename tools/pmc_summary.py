"""Per-kernel mean of rocprofv3 --pmc counter_collection csv files (development aid).
usage: python tools/pmc_summary.py DIR [name-filter]"""
import collections
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if flt and flt not in name:
                continue
            key = (name[:60], r.get("Grid_Size", r.get("Grid_Size_X", "")))
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for (name, grid), cs in acc.items():
        print(f"{name} grid={grid}")
        for c, v in sorted(cs.items()):
            print(f"    {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
