"""VALU instructions per bench step and stage from a rocprofv3 --pmc run of `bench.py --roofline-only`
(SQ_INSTS_VALU = wave-instructions, summed over the chip).  Every stage of this pipeline is bound by
VALU issue (integer / packed-f16 stencils, compaction): bench.py prices each stage's measured time
against the chip's issue rate with these counts (profiles/valu.json, like traffic.json for bytes).
usage: python tools/valu.py PMC_DIR WORKLOAD OUT_JSON"""
import collections
import csv
import glob
import json
import sys

from traffic import STAGES, stamp


def per_kernel(d, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("orbfe::", "")
                acc[name].append(float(r["Counter_Value"]))
    return acc


def main():
    d, workload, out = sys.argv[1], sys.argv[2], sys.argv[3]
    valu, lds = per_kernel(d, "SQ_INSTS_VALU"), per_kernel(d, "SQ_INSTS_LDS")
    res = {}
    for st, ks in STAGES.items():
        per_step_launches = 7 if st == "resize" else 1
        nsteps = len(valu.get(ks[0], [])) / per_step_launches
        if not nsteps:
            continue
        res[st] = {"valu_inst": sum(sum(valu.get(k, [])) for k in ks) / nsteps,
                   "lds_inst": sum(sum(lds.get(k, [])) for k in ks) / nsteps, "steps_seen": nsteps}
    data = {}
    try:
        data = json.load(open(out))
    except Exception:
        pass
    data[workload] = {st: v["valu_inst"] for st, v in res.items()}
    data[workload + "_detail"] = res
    data[workload + "_meta"] = stamp()
    json.dump(data, open(out, "w"), indent=1, sort_keys=True)
    for st, v in res.items():
        print(f"{st:9s} VALU {v['valu_inst'] / 1e6:9.1f} M  LDS {v['lds_inst'] / 1e6:8.1f} M wave-instructions per step")


if __name__ == "__main__":
    main()
