"""Debug aid: host cost of one StereoFrontEnd.enqueue (Python + ctypes + the C++ enqueue's launches) for a small
batch, without synchronising (the GPU queue runs behind), and the GPU-bound step for comparison.
usage: python tools/dbg/enqueue_cost.py [--pairs 4] [--n 200]"""
import argparse
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=4)
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--lanes", type=int, default=1)
    a = ap.parse_args()
    import torch
    from pyorbslam_amd import synth
    from pyorbslam_amd.batch import StereoFrontEnd
    from pyorbslam_amd._lib import call
    dev = torch.device("cuda", 0)
    imgs = torch.from_numpy(synth.make_batch(a.pairs)).to(dev)
    st = torch.cuda.Stream(dev)
    fe = StereoFrontEnd(max_pairs=a.pairs, lanes=a.lanes)
    for _ in range(10):
        fe.enqueue(imgs, stream_ptr=st.cuda_stream)
    torch.cuda.synchronize()
    t = []
    for _ in range(a.n):
        t0 = time.perf_counter()
        fe.enqueue(imgs, stream_ptr=st.cuda_stream)
        t.append(time.perf_counter() - t0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    gpu = (time.perf_counter() - t1)
    t.sort()
    print(f"enqueue host us: p50 {t[len(t) // 2] * 1e6:.1f} p10 {t[len(t) // 10] * 1e6:.1f} p90 {t[9 * len(t) // 10] * 1e6:.1f}; "
          f"host total {sum(t) * 1e3:.2f} ms for {a.n}, GPU drain after {gpu * 1e3:.2f} ms")
    # the raw C call alone (no Python argument checks)
    import ctypes as C
    t = []
    for _ in range(a.n):
        t0 = time.perf_counter()
        call("orbfe_frontend_batch_device", fe._h, C.c_void_p(imgs.data_ptr()), fe.width * fe.height, a.pairs, 386.1448,
             718.856, C.c_void_p(st.cuda_stream))
        t.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    t.sort()
    print(f"C call host us: p50 {t[len(t) // 2] * 1e6:.1f} p10 {t[len(t) // 10] * 1e6:.1f}")


if __name__ == "__main__":
    main()
