"""How the concurrent handles of the bench step overlap, from a rocprofv3 kernel trace of `bench.py
--roofline-only`-style runs (tools/evidence.sh `ktrace`).  Takes the dispatches of one grid height (the
handle's image count, 256 for the headline's 128-pair handles), keeps the longest stretch without an idle gap (the timed steps), sweeps its time line and reports, per stage
set running at once, the share of wall time; and the share of time each stage runs alone.
usage: python tools/ktrace_overlap.py TRACE_CSV [images_per_handle]"""
import collections
import csv
import sys

STAGE = {"k_resize_rows": "resize", "k_resize_cascade": "resize", "k_detect": "detect", "k_octree_bins": "octree",
         "k_octree": "octree", "k_orb": "describe", "k_stereo": "stereo", "k_stereo_bucket": "stereo"}


def main():
    path = sys.argv[1]
    imgs = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    ev = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("orbfe::", "")
        st = STAGE.get(name)
        if st is None:
            continue
        gy = int(r["Grid_Size_Y"])
        # k_orb / k_stereo put images in x: accept them when their handle's detect grid matched
        if name in ("k_resize_rows", "k_detect") and gy != imgs:
            continue
        if name == "k_octree_bins" and int(r["Grid_Size_X"]) != 256 * imgs:
            continue
        if name == "k_orb" and int(r["Grid_Size_X"]) > 8_000_000:
            continue
        if name == "k_stereo" and gy != imgs // 2:
            continue
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), st))
    ev.sort()
    # the longest run of dispatches without an idle gap (the timed steps, between the bench's phases)
    segs, cur, end_max = [], [ev[0]], ev[0][1]
    for e in ev[1:]:
        if e[0] > end_max:
            segs.append(cur)
            cur = []
        cur.append(e)
        end_max = max(end_max, e[1])
    segs.append(cur)
    ev = max(segs, key=lambda sg: max(x[1] for x in sg) - sg[0][0])
    pts = []
    for s, e, st in ev:
        pts.append((s, 1, st))
        pts.append((e, -1, st))
    pts.sort()
    running = collections.Counter()
    share = collections.Counter()
    alone = collections.Counter()
    busy = 0
    t0 = pts[0][0]
    last = t0
    for t, d, st in pts:
        dt = t - last
        if dt > 0:
            key = "+".join(sorted(k for k, v in running.items() for _ in range(v))) or "(idle)"
            share[key] += dt
            if sum(running.values()) == 1:
                alone[next(k for k, v in running.items() if v)] += dt
            if running:
                busy += dt
        running[st] += d
        if running[st] == 0:
            del running[st]
        last = t
    span = last - t0
    gaps = []
    end_max = ev[0][1]
    for s_, e_, st in ev[1:]:
        if s_ > end_max:
            gaps.append((s_ - end_max, end_max - t0, st))
        end_max = max(end_max, e_)
    gaps.sort(reverse=True)
    print("largest idle gaps (us, at ms, next stage):", [(round(g / 1e3, 1), round(a / 1e6, 2), st) for g, a, st in gaps[:12]])
    print(f"idle gaps: {len(gaps)}, total {sum(g for g, _, _ in gaps) / 1e6:.3f} ms; below 50 us: "
          f"{sum(g for g, _, _ in gaps if g < 50e3) / 1e6:.3f} ms")
    print(f"{len(ev)} dispatches, span {span / 1e6:.3f} ms, some kernel running {busy / span:.3f}")
    print("stage alone (share of span):", {k: round(v / span, 3) for k, v in alone.most_common()})
    print("concurrent stage sets, top 25 (share of span):")
    for k, v in share.most_common(25):
        print(f"  {v / span:6.3f}  {k}")


if __name__ == "__main__":
    main()
