"""cpu_baseline's all-cores leg at several process counts on the GPU box: with the job's
cgroup granting 16 CPUs' worth of time (cpu.max 1600000 / 100000) while its affinity mask shows 256 hardware
threads, more than 16 processes share the same 16 CPUs.  usage: python tools/cpu_quota_probe.py [procs ...]"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402

if __name__ == "__main__":
    print(json.dumps(bench.job_cpus()), flush=True)
    for p in [int(a) for a in sys.argv[1:]] or [16, 32, 64]:
        r = bench.cpu_baseline(2, 1241, 376, 2000, p)
        print(json.dumps({"procs": p, "pairs_per_s": round(r["value"], 2), "value_1core": round(r["value_1core"], 3)}),
              flush=True)
