"""HBM traffic per bench step and stage from rocprofv3 --pmc runs of bench.py (FETCH_SIZE and WRITE_SIZE
in separate passes, as MI355X_MICROARCH.md prescribes).  FETCH_SIZE / WRITE_SIZE are in KiB per
dispatch; FETCH_SIZE is doubled (gfx950 tallies 128-B memory-side read requests at 64 B).  These
kernels use dword/dwordx2/byte loads, for which the guide's x2 calibration is not established, so the
raw and corrected values are both kept.
usage: python tools/traffic.py PMC_DIR WORKLOAD OUT_JSON [steps]"""
import collections
import csv
import glob
import json
import sys
from pathlib import Path

STAGES = {"resize": ["k_resize_rows", "k_resize"], "detect": ["k_detect"], "octree": ["k_octree_bins", "k_octree"],
          "describe": ["k_orb"], "stereo": ["k_stereo", "k_stereo_bucket"]}  # (buckets inside k_orb since round 5)


def stamp() -> dict:
    """Build id of the library the PMC runs measured (the in-tree build that travelled to the GPU box) and
    the git revision: bench.py uses an entry only when the build id matches the library it loads."""
    import subprocess
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    from pyorbslam_amd import _lib
    try:
        rev = subprocess.check_output(["git", "rev-parse", "--short=12", "HEAD"], cwd=Path(__file__).resolve().parents[1],
                                      text=True).strip()
        dirty = subprocess.call(["git", "diff", "--quiet", "HEAD", "--", "pyorbslam_amd/csrc", "include"],
                                cwd=Path(__file__).resolve().parents[1]) != 0
    except Exception:
        rev, dirty = "unknown", False
    return {"build_id": _lib.build_id(), "git_rev": rev + ("+uncommitted-kernel-edits" if dirty else "")}


def per_kernel(d, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("orbfe::", "")
                acc[name].append(float(r["Counter_Value"]) * 1024.0)
    return acc


def main():
    d, workload, out = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch, write = per_kernel(d, "FETCH_SIZE"), per_kernel(d, "WRITE_SIZE")
    res = {}
    for st, ks in STAGES.items():
        # bytes per step: all dispatches of the stage's kernels / number of steps (dispatches of the
        # first kernel / its launches per step)
        per_step_launches = 7 if st == "resize" else 1
        nsteps = len(fetch.get(ks[0], [])) / per_step_launches
        if not nsteps:
            continue
        f = sum(sum(fetch.get(k, [])) for k in ks) / nsteps
        w = sum(sum(write.get(k, [])) for k in ks) / nsteps
        res[st] = {"fetch_raw_bytes": f, "write_bytes": w, "bytes": 2 * f + w, "steps_seen": nsteps}
    data = {}
    try:
        data = json.load(open(out))
    except Exception:
        pass
    data[workload] = {st: v["bytes"] for st, v in res.items()}
    data[workload + "_detail"] = res
    data[workload + "_meta"] = stamp()
    json.dump(data, open(out, "w"), indent=1, sort_keys=True)
    for st, v in res.items():
        print(f"{st:9s} fetch(raw) {v['fetch_raw_bytes'] / 1e6:9.1f} MB  write {v['write_bytes'] / 1e6:9.1f} MB  "
              f"corrected total {v['bytes'] / 1e6:9.1f} MB per step")


if __name__ == "__main__":
    main()
