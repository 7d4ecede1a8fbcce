"""Per-kernel dispatch statistics from a rocprofv3 --kernel-trace csv, grouped by (kernel, grid size).

The default bench command launches every kernel twice over: 4 concurrent handles of 64 pairs (128-image
grids) in the timed region, then the standalone pass of 256 pairs on one stream (512-image grids) that
the JSON line's roofline comes from; grouping by grid size separates the two.
usage: python tools/kernel_table.py run_kernel_trace.csv OUT.md"""
import collections
import csv
import sys
from pathlib import Path


def main(src, dst):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(src)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("orbfe::", "")
        grid = f"{r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
        acc[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    total = sum(sum(v) for v in acc.values())
    lines = ["| kernel | grid (threads x, y, z) | calls | avg us | min us | max us | total us | % |",
             "|---|---|---|---|---|---|---|---|"]
    for (name, grid), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| `{name[:60]}` | {grid} | {len(v)} | {sum(v) / len(v):.1f} | {min(v):.1f} | {max(v):.1f} | "
                     f"{sum(v):.1f} | {100 * sum(v) / total:.1f} |")
    Path(dst).write_text("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
