"""Condense tools/ab.sh output: per library the bench values of every round (mean, spread) and, when
PMC passes exist, per env step of mmx_env_step_kernel: VALU instructions, active-lane fraction,
LDS bank-conflict cycles per LDS-active cycle.  Writes <dir>/report.json and prints it."""
import csv
import glob
import json
import os
import sys

KERNEL = "mmx_env_step_kernel"


def pmc(d):
    tot, disp = {}, set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f, newline="")):
            if KERNEL not in r.get("Kernel_Name", ""):
                continue
            disp.add(r.get("Dispatch_Id"))
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return tot, len(disp)


def main(out):
    runs = {}
    for ln in open(os.path.join(out, "ab.txt")):
        name, js = ln.split(" ", 1)
        d = json.loads(js)
        runs.setdefault(name, []).append(d)
    rep = {}
    for name, ds in runs.items():
        v = [d["value"] for d in ds]
        r = {"values": [round(x) for x in v], "mean": sum(v) / len(v), "kernel_ms": [round(d["roofline"]["kernel_ms"], 3) for d in ds]}
        pdir = os.path.join(out, f"pmc_{name}")
        if os.path.isdir(pdir):
            t, n = pmc(pdir)
            d0 = ds[0]
            env_steps = d0["config"]["envs_per_gpu"] * (d0["steps"] + d0["warmup"])
            r["pmc"] = {"dispatches": n,
                        "valu_per_env_step": t.get("SQ_INSTS_VALU", 0) / env_steps,
                        "active_lanes": t.get("SQ_THREAD_CYCLES_VALU", 0) / max(64 * t.get("SQ_ACTIVE_INST_VALU", 1), 1),
                        "lds_conflict_per_lds_cycle": t.get("SQ_LDS_BANK_CONFLICT", 0) / max(t.get("SQ_ACTIVE_INST_LDS", 1), 1),
                        "lds_insts_per_env_step": t.get("SQ_INSTS_LDS", 0) / env_steps,
                        "valu_issue": t.get("SQ_ACTIVE_INST_VALU", 0) / max(t.get("SQ_WAVE_CYCLES", 1), 1),
                        "raw": t}
        rep[name] = r
    base = rep.get("libmmx", {}).get("mean")
    for name, r in rep.items():
        if base:
            r["vs_product"] = r["mean"] / base - 1
    json.dump(rep, open(os.path.join(out, "report.json"), "w"), indent=1)
    for name, r in rep.items():
        p = r.get("pmc", {})
        print(f"{name:24s} mean {r['mean']:.0f} ({'%+.2f %%' % (100 * r.get('vs_product', 0))}) {r['values']}"
              + (f" valu/step {p['valu_per_env_step']:.0f} lanes {p['active_lanes']:.3f} ldsconf {p['lds_conflict_per_lds_cycle']:.3f}"
                 if p else ""))


if __name__ == "__main__":
    main(sys.argv[1])
