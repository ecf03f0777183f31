"""Condense rocprofv3 CSV output (tools/profile.sh) into committed evidence under profiles/.

- profiles/<round>_<workload>_kernel_stats.csv : rocprofv3 --stats summary of the traced bench run
- profiles/<round>_<workload>_bench_trace.json : the bench JSON line printed under the tracer
- profiles/pmc_<workload>.json (+ a <round>_ copy): per env step of mmx_env_step_kernel over the
  timed window's dispatches (the last ones of each pass), tagged with the configuration:
    * HBM-side bytes: FETCH_SIZE x2 (gfx950: it tallies 128-B read requests at 64 B,
      MI355X_MICROARCH.md §HBM) + WRITE_SIZE, KB -> bytes, each counter from its own pass;
    * VALU issue: SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES per wave x resident waves per SIMD.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil

KERNEL = "mmx_env_step_kernel"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rows(pattern):
    out = []
    for f in sorted(glob.glob(pattern, recursive=True)):
        with open(f, newline="") as fh:
            out.extend(csv.DictReader(fh))
    return out


def per_dispatch(prof_dir: str, counters: list[str]) -> list[dict]:
    """[{counter: value}] per dispatch of KERNEL, in dispatch order."""
    per = {}
    for r in _rows(os.path.join(prof_dir, "**", "*counter_collection.csv")):
        if KERNEL not in r.get("Kernel_Name", "") or r.get("Counter_Name") not in counters:
            continue
        d = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
        per.setdefault(d, {}).setdefault(r["Counter_Name"], 0.0)
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        raise SystemExit(f"no {counters} rows for {KERNEL} under {prof_dir}")
    return [per[d] for d in sorted(per)]


def timed_mean(rows: list[dict], n_last: int) -> dict:
    rows = rows[-n_last:]
    return {k: sum(r.get(k, 0.0) for r in rows) / len(rows) for k in rows[0]}


EXT_A = ["SQ_WAVE_CYCLES", "SQ_WAVES", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH",
         "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"]
EXT_B = ["SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC", "SQ_INST_CYCLES_SALU", "SQ_WAIT_INST_LDS",
         "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_ACTIVE_INST_VALU"]


def extended_sq(prof: str, n_timed: int, config: dict, rnd: str) -> dict | None:
    """The two extended SQ passes (profile.sh sqx_a / sqx_b) per dispatch and per wave quad-cycle
    (each counter over its own pass's SQ_WAVE_CYCLES); None when the passes are missing."""
    da, db = os.path.join(prof, "sqx_a"), os.path.join(prof, "sqx_b")
    if not (os.path.isdir(da) and os.path.isdir(db)):
        return None
    a = timed_mean(per_dispatch(da, EXT_A), n_timed)
    b = timed_mean(per_dispatch(db, EXT_B), n_timed)
    per = dict(a)
    per.update({k: v for k, v in b.items() if k != "SQ_WAVE_CYCLES"})
    norm = {k: round(v / a["SQ_WAVE_CYCLES"], 4) for k, v in a.items()}
    norm.update({k: round(v / b["SQ_WAVE_CYCLES"], 4) for k, v in b.items() if k != "SQ_WAVE_CYCLES"})
    return {"kernel": KERNEL, "round": rnd, "config": config, "timed_dispatches": n_timed,
            "per_dispatch": per, "per_wave_quad_cycle": norm,
            "reading": (f"per wave and quad-cycle: any instruction issued {norm['SQ_ACTIVE_INST_ANY']:.2f} (VALU "
                        f"{norm['SQ_ACTIVE_INST_VALU']:.2f}, SALU {norm['SQ_INSTS_SALU']:.2f}, LDS "
                        f"{norm['SQ_INSTS_LDS']:.3f}, branch {norm['SQ_INSTS_BRANCH']:.3f}); a wave can issue ~0.94 VALU "
                        "per quad-cycle (profiles/r05_valu_issue_calibration.json)")}



def valu_ceiling(waves_per_simd: float):
    """What a SIMD (and one of its waves) can issue at this many resident waves per SIMD, in the units
    of SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES: the calibration kernel's measured issue (8 independent FMA
    chains per wave, profiles/r05_valu_issue_calibration.json) interpolated over 1-4 waves per SIMD."""
    import numpy as np

    cal = json.load(open(os.path.join(REPO, "profiles", "r05_valu_issue_calibration.json")))
    rows = sorted((r["waves_per_simd"], r["sq_active_inst_valu_per_wave_quad_cycle"], r["sq_valu_per_simd_quad_cycle"])
                  for r in cal["scalar_v_fma_f32"] if r["chains"] == 8)
    w = [r[0] for r in rows]
    return float(np.interp(waves_per_simd, w, [r[1] for r in rows])), float(np.interp(waves_per_simd, w, [r[2] for r in rows]))


def valu_reading(per_wave: float, waves_per_simd: float) -> dict:
    """VALU issue of the kernel against the calibrated ceiling: 'latency' below 0.6 of it."""
    cw, cs = valu_ceiling(waves_per_simd)
    frac = per_wave / cw
    return {"valu_issue_per_wave": per_wave, "waves_per_simd": waves_per_simd, "valu_issue_per_simd": per_wave * waves_per_simd,
            "issue_ceiling_per_wave": cw, "issue_ceiling_per_simd": cs, "frac_of_ceiling": frac,
            "bound": "latency" if frac < 0.6 else "valu-issue",
            "units": "SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (instructions per quad-cycle); ceiling: "
                     "profiles/r05_valu_issue_calibration.json at the kernel's waves per SIMD"}

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r03")
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--prof", required=True)
    ap.add_argument("--timed-steps", type=int, default=64)
    a = ap.parse_args()
    dst = os.path.join(REPO, "profiles")
    os.makedirs(dst, exist_ok=True)
    tag = f"{a.round}_{a.workload}"
    stats = glob.glob(os.path.join(a.prof, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(dst, f"{tag}_kernel_stats.csv"))
    line = None
    for name in ("bench_trace", "bench_fetch", "bench_write", "bench_sq"):
        log = os.path.join(a.prof, f"{name}.log")
        lines = [ln for ln in open(log) if ln.startswith("{")] if os.path.exists(log) else []
        if lines:
            if name == "bench_trace":
                open(os.path.join(dst, f"{tag}_bench_trace.json"), "w").write(lines[-1])
            line = line or json.loads(lines[-1])
    rf = line["roofline"]
    lanes, spl, epl = rf["concurrent_launches"], rf["env_steps_per_launch"], rf["envs_per_launch"]
    n_timed = lanes * int(round(a.timed_steps / spl))  # dispatches of the timed window (the last ones)
    unit = epl * spl  # env steps per dispatch (mean: launch lengths differ by at most one step)
    fetch = timed_mean(per_dispatch(os.path.join(a.prof, "fetch"), ["FETCH_SIZE"]), n_timed)["FETCH_SIZE"]
    write = timed_mean(per_dispatch(os.path.join(a.prof, "write"), ["WRITE_SIZE"]), n_timed)["WRITE_SIZE"]
    sq_names = ["SQ_WAVE_CYCLES", "SQ_WAVES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU",
                "SQ_ACTIVE_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_ANY"]
    sq = timed_mean(per_dispatch(os.path.join(a.prof, "sq"), sq_names), n_timed)
    lanes_dir = os.path.join(a.prof, "lanes")
    lane_util = None
    if os.path.isdir(lanes_dir):
        ln = timed_mean(per_dispatch(lanes_dir, ["SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU"]), n_timed)
        lane_util = ln["SQ_THREAD_CYCLES_VALU"] / max(64.0 * ln["SQ_ACTIVE_INST_VALU"], 1.0)
    # resident waves per SIMD: the 128-row layout runs one wave per env, at most 12 envs per CU (12,640 B
    # of LDS per env in 1,280-byte blocks; r05: 11); the 192-row layout two (the env wave and its helper),
    # at most 4 envs per CU
    helper = int(line["config"].get("step_kernel_lds_rows", 128)) == 192
    per_cu = float(os.environ.get("MMX_ENVS_PER_CU", "4" if helper else "12"))
    waves_per_simd = min(per_cu * 256.0, float(line["config"]["envs_per_gpu"])) * (2.0 if helper else 1.0) / 1024.0
    per_wave = sq["SQ_ACTIVE_INST_VALU"] / sq["SQ_WAVE_CYCLES"]
    hbm = 2.0 * fetch * 1024.0 + write * 1024.0
    rec = {
        "kernel": KERNEL, "round": a.round, "source": f"profiles/{tag}_pmc.json (tools/profile.sh)",
        "config": {"workload": line["config"]["workload"].split(":")[0].lower(), "envs_per_gpu": line["config"]["envs_per_gpu"],
                   "env_steps_per_launch": spl, "lanes": lanes},
        "timed_dispatches": n_timed, "env_steps_per_dispatch": unit,
        "fetch_size_kb_raw": fetch, "write_size_kb": write,
        "hbm_bytes_per_dispatch": hbm, "hbm_bytes_per_env_step": hbm / unit,
        "fetch_bytes_per_env_step": 2.0 * fetch * 1024.0 / unit, "write_bytes_per_env_step": write * 1024.0 / unit,
        "sq_per_dispatch": sq,
        "valu": {**valu_reading(per_wave, waves_per_simd), "active_inst_valu_per_wave_cycle": per_wave,
                 "valu_insts_per_env_step": sq["SQ_INSTS_VALU"] / unit,
                 "lds_bank_conflict_per_lds_active": sq["SQ_LDS_BANK_CONFLICT"] / max(sq["SQ_ACTIVE_INST_LDS"], 1.0),
                 "wait_any_per_wave_cycle": sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"],
                 # mean fraction of the 64 lanes active per VALU instruction (rocprofiler's
                 # AvgNumActiveThreads / 64 for gfx950); None when the pass is missing
                 "active_lane_fraction": lane_util},
        "note": "FETCH_SIZE x2 (gfx950 wide-read tally, MI355X_MICROARCH.md §HBM); dword-per-lane reads uncalibrated; "
                "Infinity-Cache hits are counted by these memory-side counters",
    }
    if rec["config"]["workload"] not in ("c2", "c3", "c5"):
        rec["config"]["workload"] = a.workload
    ext = extended_sq(a.prof, n_timed, rec["config"], a.round)
    if ext:
        json.dump(ext, open(os.path.join(dst, f"{tag}_sq_extended.json"), "w"), indent=1)
    json.dump(rec, open(os.path.join(dst, f"pmc_{a.workload}.json"), "w"), indent=1)
    json.dump(rec, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1)
    print(json.dumps({k: rec[k] for k in ("hbm_bytes_per_env_step", "valu")}))


if __name__ == "__main__":
    main()
