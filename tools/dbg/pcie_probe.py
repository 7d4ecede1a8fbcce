"""Host <-> device copy rates with pinned memory (development aid for bench.py's host_fed line): the 512-pair
image batch H2D alone as 1 / 2 / 4 chunks on as many streams, the records D2H alone, and both at once.
usage: python tools/dbg/pcie_probe.py [--mb 478]"""
import argparse
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=478)
    ap.add_argument("--out-mb", type=int, default=126)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, m = a.mb << 20, a.out_mb << 20
    hin = torch.empty(n, dtype=torch.uint8).pin_memory()
    din = torch.empty(n, dtype=torch.uint8, device=dev)
    dout = torch.empty(m, dtype=torch.uint8, device=dev)
    hout = torch.empty(m, dtype=torch.uint8).pin_memory()
    streams = [torch.cuda.Stream(dev) for _ in range(4)]

    def run(k, h2d=True, d2h=False, reps=5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            if h2d:
                step = n // k
                for i in range(k):
                    with torch.cuda.stream(streams[i]):
                        din[i * step:(i + 1) * step].copy_(hin[i * step:(i + 1) * step], non_blocking=True)
            if d2h:
                with torch.cuda.stream(streams[3]):
                    hout.copy_(dout, non_blocking=True)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    run(1)
    for k in (1, 2, 4):
        dt = run(k)
        print(f"H2D {a.mb} MB as {k} chunk(s): {dt * 1e3:.2f} ms  {n / dt / 1e9:.1f} GB/s", flush=True)
    dt = run(1, h2d=False, d2h=True)
    print(f"D2H {a.out_mb} MB: {dt * 1e3:.2f} ms  {m / dt / 1e9:.1f} GB/s", flush=True)
    dt = run(2, h2d=True, d2h=True)
    print(f"H2D {a.mb} MB (2 chunks) + D2H {a.out_mb} MB together: {dt * 1e3:.2f} ms  H2D-equivalent "
          f"{n / dt / 1e9:.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
