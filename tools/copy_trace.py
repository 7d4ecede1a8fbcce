"""Summary of a rocprofv3 --kernel-trace --memory-copy-trace run (tools/host_fed_trace.py): per direction the
copies' count, bytes, summed duration and GB/s while copying; the span of the traced window; the share of that
span during which a host->device copy is in flight, during which any kernel runs, and both at once.
usage: python tools/copy_trace.py TRACE_DIR [--last-h2d 32] [--h2d-bytes 119453696] [--d2h-bytes 23670784]
(rocprofv3's memory-copy records carry no size: --h2d-bytes is the host-fed chunk, 128 pairs x 2 x 1241 x 376;
the window is the last --last-h2d host->device copies, i.e. the timed steps, to the end of the last kernel)"""
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
    ap.add_argument("--last-h2d", type=int, default=32)
    ap.add_argument("--h2d-bytes", type=int, default=2 * 128 * 1241 * 376)
    ap.add_argument("--d2h-bytes", type=int, default=128 * 184928)
    a = ap.parse_args()
    kern, cop, blit = [], [], []
    for f in glob.glob(f"{a.trace}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            iv = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
            # ROCclr moves device->pinned-host copies with a blit kernel: count those as the D2H leg
            (blit if r["Kernel_Name"].startswith("__amd_rocclr_copy") else kern).append(iv)
    for f in glob.glob(f"{a.trace}/**/*memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            d = r.get("Direction", r.get("Kind", "?"))
            cop.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), d, int(r.get("Bytes", r.get("Size", 0)))))
    if not kern or not cop:
        raise SystemExit("no kernel or copy records")
    h2d = sorted(c for c in cop if "HOST_TO_DEVICE" in c[2])
    if a.last_h2d and len(h2d) >= a.last_h2d:
        t0 = h2d[-a.last_h2d][0]
        cop = [(s_, e_, d_, b_ or (a.h2d_bytes if "HOST_TO_DEVICE" in d_ else 0)) for s_, e_, d_, b_ in cop]
    else:
        t0 = min(k[0] for k in kern) + int(a.skip_first_s * 1e9)
    kern = [k for k in kern if k[0] >= t0]
    cop = [c for c in cop if c[0] >= t0]
    span = max(max(k[1] for k in kern), max(c[1] for c in cop)) - t0
    K = union(kern)
    print(f"window {span / 1e6:.3f} ms, kernel-busy (orbfe kernels) {sum(e - s for s, e in K) / span:.3f} of it")
    blit = [b for b in blit if b[0] >= t0]
    if blit:
        B = union(blit)
        durs = sorted((e - s) / 1e3 for s, e in blit)
        bb = a.d2h_bytes * len(blit)
        print(f"blit copy kernels (__amd_rocclr_copyBuffer, the D2H record leg): {len(blit)}, per-kernel us p50 "
              f"{durs[len(durs) // 2]:.1f}, in flight {sum(e - s for s, e in B) / span:.3f} of the window, "
              f"{bb / max(sum(e - s for s, e in B), 1):.2f} GB/s while in flight at --d2h-bytes each, "
              f"overlapping orbfe kernels {inter(B, K) / max(sum(e - s for s, e in B), 1):.3f}")
    for d in sorted({c[2] for c in cop}):
        cs = [c for c in cop if c[2] == d]
        durs = sorted((c[1] - c[0]) / 1e3 for c in cs)
        print(f"{d}: per-copy us p50 {durs[len(durs) // 2]:.1f} min {durs[0]:.1f} max {durs[-1]:.1f}")
        U = union([(c[0], c[1]) for c in cs])
        busy = sum(e - s for s, e in U)
        b = sum(c[3] for c in cs)
        print(f"{d}: {len(cs)} copies, {b / 1e6:.1f} MB, in flight {busy / span:.3f} of the window, "
              f"{b / max(busy, 1):.2f} GB/s while in flight, overlapping kernels {inter(U, K) / max(busy, 1):.3f}")


if __name__ == "__main__":
    main()
