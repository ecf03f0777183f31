"""Condense rocprofv3 CSV output into committed evidence under profiles/.

- profiles/<round>_kernel_stats.csv : rocprofv3 --stats summary of the bench run (copied)
- profiles/<round>_bench_trace.json : the bench JSON line printed under the tracer
- profiles/pmc_traffic.json         : HBM-side bytes per launch of mmx_env_step_kernel from
  the FETCH_SIZE and WRITE_SIZE passes (KB -> bytes; FETCH_SIZE doubled per the gfx950 note in
  MI355X_MICROARCH.md §HBM: it tallies 128-B read requests at 64 B), averaged over dispatches.
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
    for f in glob.glob(pattern, recursive=True):
        with open(f, newline="") as fh:
            out.extend(csv.DictReader(fh))
    return out


def counter_per_dispatch(prof_dir: str, counter: str) -> tuple[float, int]:
    rows = _rows(os.path.join(prof_dir, "**", "*counter_collection.csv"))
    per = {}
    for r in rows:
        if KERNEL not in r.get("Kernel_Name", "") or r.get("Counter_Name") != counter:
            continue
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        per[d] = per.get(d, 0.0) + float(r["Counter_Value"])
    if not per:
        raise SystemExit(f"no {counter} rows for {KERNEL} under {prof_dir}")
    return sum(per.values()) / len(per), len(per)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r01")
    ap.add_argument("--prof", default=os.path.join(REPO, "gpurun_out", "prof"))
    a = ap.parse_args()
    dst = os.path.join(REPO, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(a.prof, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(dst, f"{a.round}_kernel_stats.csv"))
    log = os.path.join(a.prof, "bench_trace.log")
    if os.path.exists(log):
        lines = [ln for ln in open(log) if ln.startswith("{")]
        if lines:
            open(os.path.join(dst, f"{a.round}_bench_trace.json"), "w").write(lines[-1])
    fetch_kb, nf = counter_per_dispatch(os.path.join(a.prof, "fetch"), "FETCH_SIZE")
    write_kb, nw = counter_per_dispatch(os.path.join(a.prof, "write"), "WRITE_SIZE")
    rec = {
        "kernel": KERNEL, "round": a.round,
        "fetch_size_kb_raw": fetch_kb, "write_size_kb": write_kb, "dispatches": [nf, nw],
        "fetch_bytes_corrected": 2.0 * fetch_kb * 1024.0, "write_bytes": write_kb * 1024.0,
        "bytes_per_launch": 2.0 * fetch_kb * 1024.0 + write_kb * 1024.0,
        "note": "FETCH_SIZE x2 (gfx950 wide-read tally); dword-per-lane reads are uncalibrated",
    }
    json.dump(rec, open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
    json.dump(rec, open(os.path.join(dst, f"{a.round}_pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
