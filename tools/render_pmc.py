"""Condense the render_pmc recipe of tools/gpu.sh: mean SQ counters per mmx_render_kernel dispatch (the last
`--last` dispatches) and per workgroup / per pixel -> profiles/<round>_render_pmc.json.  Diagnostic."""
import argparse
import csv
import glob
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))



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
    ap.add_argument("--prof", default=os.path.join(REPO, "gpurun_out", "rpmc"))
    ap.add_argument("--last", type=int, default=32)
    ap.add_argument("--wg-per-dispatch", type=int, default=8192 * 2)  # envs x cameras (128^2: both bands in one workgroup)
    ap.add_argument("--px-per-dispatch", type=int, default=8192 * 2 * 128 * 128)
    ap.add_argument("--lanes", type=int, default=1)  # the C5 rollout's lanes (bench.py matches on it)
    a = ap.parse_args()
    per = {}
    for f in glob.glob(os.path.join(a.prof, "**", "*counter_collection.csv"), recursive=True):
        pas = os.path.relpath(f, a.prof).split(os.sep)[0]
        for r in csv.DictReader(open(f, newline="")):
            if "mmx_render_kernel" not in r.get("Kernel_Name", ""):
                continue
            # launches of the configured shape only (r05: one render of all 8192 envs x 2 cameras per
            # step, the same grid as the bench's isolated render timing through mmx_forward)
            if int(r.get("Grid_Size") or 0) != a.wg_per_dispatch * 512:
                continue
            d = (pas, int(r.get("Dispatch_Id") or r.get("Correlation_Id")))
            per.setdefault(d, {}).setdefault(r["Counter_Name"], 0.0)
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for pas in sorted({p for p, _ in per}):
        ds = sorted(d for d in per if d[0] == pas)[-a.last:]
        for k in per[ds[0]]:
            out[k] = sum(per[d][k] for d in ds) / len(ds)
    res = {"kernel": "mmx_render_kernel", "source": f"tools/render_pmc.sh (C5, 128^2, {a.wg_per_dispatch // 2} envs per dispatch)",
           "per_dispatch": out,
           "per_workgroup": {k: v / a.wg_per_dispatch for k, v in out.items()},
           "valu_issue_per_wave_cycle": out.get("SQ_ACTIVE_INST_VALU", 0) / max(out.get("SQ_WAVE_CYCLES", 1), 1),
           "valu_insts_per_px": out.get("SQ_INSTS_VALU", 0) * 64 / a.px_per_dispatch}
    # what bench.py's C5 line cites (its `render.valu`), tagged with the configuration measured
    waves_per_simd = 4  # 512-lane workgroups (8 waves), two per CU (LDS), 4 SIMDs
    res["config"] = {"workload": "render", "envs_per_gpu": 8192, "env_steps_per_launch": 1, "lanes": a.lanes}
    res["valu"] = {**valu_reading(res["valu_issue_per_wave_cycle"], waves_per_simd), "valu_insts_per_px": res["valu_insts_per_px"],
                   "active_inst_valu_per_wave_cycle": res["valu_issue_per_wave_cycle"],
                   "wait_any_per_wave_cycle": out.get("SQ_WAIT_ANY", 0) / max(out.get("SQ_WAVE_CYCLES", 1), 1),
                   "source": f"profiles/{a.round}_render_pmc.json"}
    dst = os.path.join(REPO, "profiles", f"{a.round}_render_pmc.json")
    json.dump(res, open(dst, "w"), indent=1)
    json.dump(res, open(os.path.join(REPO, "profiles", "pmc_render.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
