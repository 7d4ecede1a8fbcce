"""Summary of a rocprofv3 --kernel-trace --memory-copy-trace run (tools/host_fed_trace.py): per direction the
copies' count, bytes, summed duration and GB/s while copying; the span of the traced window; the share of that
span during which a host->device copy is in flight, during which any kernel runs, and both at once.
usage: python tools/copy_trace.py TRACE_DIR [--skip-first-s 0.0]"""
import argparse
import csv
import glob


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def inter(a, b):
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip-first-s", type=float, default=0.0)
    a = ap.parse_args()
    kern, cop = [], []
    for f in glob.glob(f"{a.trace}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            kern.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for f in glob.glob(f"{a.trace}/**/*memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            d = r.get("Direction", r.get("Kind", "?"))
            cop.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), d, int(r.get("Bytes", r.get("Size", 0)))))
    if not kern or not cop:
        raise SystemExit("no kernel or copy records")
    t0 = min(k[0] for k in kern) + int(a.skip_first_s * 1e9)
    kern = [k for k in kern if k[0] >= t0]
    cop = [c for c in cop if c[0] >= t0]
    span = max(max(k[1] for k in kern), max(c[1] for c in cop)) - t0
    K = union(kern)
    print(f"window {span / 1e6:.3f} ms, kernel-busy {sum(e - s for s, e in K) / span:.3f} of it")
    for d in sorted({c[2] for c in cop}):
        cs = [c for c in cop if c[2] == d]
        U = union([(c[0], c[1]) for c in cs])
        busy = sum(e - s for s, e in U)
        b = sum(c[3] for c in cs)
        print(f"{d}: {len(cs)} copies, {b / 1e6:.1f} MB, in flight {busy / span:.3f} of the window, "
              f"{b / max(busy, 1):.2f} GB/s while in flight, overlapping kernels {inter(U, K) / max(busy, 1):.3f}")


if __name__ == "__main__":
    main()
