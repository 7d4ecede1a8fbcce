"""Workload for a rocprofv3 kernel + memory-copy trace of bench.py's host-fed step: the
512 KITTI pairs streamed from pinned host memory every step (images H2D on a copy stream, the batch, compact
records D2H), `--steps` steps after 3 untimed ones, nothing else.
usage: rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d OUT -o run -- \
           python tools/host_fed_trace.py [--steps 8] [--records 1]
Analyse with tools/copy_trace.py OUT."""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=512)
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--records", type=int, default=1)
    a = ap.parse_args()
    import torch
    import bench
    from pyorbslam_amd import synth
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    host = synth.make_batch(a.pairs, seed0=0)
    images = torch.from_numpy(host).to(dev)
    sh = bench.Shard(images, a.pairs, a.streams, dev, 1241, 376, 2000)
    r = bench.host_fed(sh, host, dev, 1, a.steps, 3, records=bool(a.records))
    print(r, flush=True)


if __name__ == "__main__":
    main()
