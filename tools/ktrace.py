"""Per-dispatch durations from a rocprofv3 --kernel-trace csv (development aid).
usage: python tools/ktrace.py gpurun_out/kt/run_kernel_trace.csv [name-filter ...]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    flt = sys.argv[2:]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    prev = None
    for r in rows:
        if flt and not any(f in r["Kernel_Name"] for f in flt):
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev else 0.0
        prev = e
        print(f"{r['Kernel_Name'][:40]:40s} grid {r['Grid_Size_X']:>7s}x{r['Grid_Size_Y']:>4s} wg {r['Workgroup_Size_X']:>4s} "
              f"lds {r['LDS_Block_Size']:>6s} vgpr {r['VGPR_Count']:>4s}  {(e - s) / 1e3:8.1f} us  gap {gap:7.1f}")


if __name__ == "__main__":
    main()
