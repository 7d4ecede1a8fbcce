"""VALU instructions per bench step and stage from a rocprofv3 --pmc run of `bench.py --roofline-only`
(SQ_INSTS_VALU = wave-instructions, summed over the chip).  Every stage of this pipeline is bound by
VALU issue (integer / packed-f16 stencils, compaction): bench.py prices each stage's measured time
against the chip's issue rate with these counts (profiles/valu.json, like traffic.json for bytes).
usage: python tools/valu.py PMC_DIR WORKLOAD OUT_JSON [BUSY_PMC_DIR]

BUSY_PMC_DIR (optional): a pass with SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE over the
same command.  Per stage it adds the VALU-busy fraction from busy cycles rather than from a class peak:
  valu_busy = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)   (SQ_* count quad-cycles summed
  over waves; GRBM_GUI_ACTIVE is summed over the 8 XCDs, MI355X_MICROARCH.md), the issue-stall share
  SQ_WAIT_INST_ANY / SQ_BUSY_CYCLES, and the effective clock GRBM_GUI_ACTIVE / 8 / the stage's dispatch time
  is left to the reader (bench.py has the times).  Stored as <workload>["busy"][stage]."""
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
    if len(sys.argv) > 4:
        bd = sys.argv[4]
        act, busy, wait, gui = (per_kernel(bd, c) for c in ("SQ_ACTIVE_INST_VALU", "SQ_BUSY_CYCLES",
                                                             "SQ_WAIT_INST_ANY", "GRBM_GUI_ACTIVE"))
        busy_out = {}
        for st, ks in STAGES.items():
            a = sum(sum(act.get(k, [])) for k in ks)
            g = sum(sum(gui.get(k, [])) for k in ks)
            b = sum(sum(busy.get(k, [])) for k in ks)
            w = sum(sum(wait.get(k, [])) for k in ks)
            if g <= 0:
                continue
            busy_out[st] = {"valu_busy": round(4 * a / (1024 * g / 8), 4),
                            "wait_inst_any_over_busy": round(w / b, 4) if b else None,
                            "SQ_ACTIVE_INST_VALU": a, "SQ_BUSY_CYCLES": b, "SQ_WAIT_INST_ANY": w, "GRBM_GUI_ACTIVE": g,
                            "dispatches": len(gui.get(ks[0], []))}
            print(f"{st:9s} VALU-busy {busy_out[st]['valu_busy']:.3f}  wait_inst/busy "
                  f"{busy_out[st]['wait_inst_any_over_busy']}")
        data[workload]["busy"] = busy_out
    data[workload + "_detail"] = res
    data[workload + "_meta"] = stamp()
    json.dump(data, open(out, "w"), indent=1, sort_keys=True)
    for st, v in res.items():
        print(f"{st:9s} VALU {v['valu_inst'] / 1e6:9.1f} M  LDS {v['lds_inst'] / 1e6:8.1f} M wave-instructions per step")


if __name__ == "__main__":
    main()
