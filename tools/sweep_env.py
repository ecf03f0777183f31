"""Interleaved A/B of run-time settings (environment variables read by libmmx.so at create / launch)
on one bench configuration: every setting runs once per round, rounds interleaved, and the report
gives each setting's median line value and its windows.  Run on the GPU box from the repo root:
    python tools/sweep_env.py --bench-args "--steps 20 --warmup 5" --rounds 2 "" "MMX_PLAN=1,1" ...
("" = the library's defaults).  Writes gpurun_out/sweep_env.json.  Experiment infrastructure."""
import argparse
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bench-args", default="--steps 20 --warmup 5")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "sweep_env.json"))
    ap.add_argument("settings", nargs="+")
    a = ap.parse_args()
    res = {s: [] for s in a.settings}
    for r in range(a.rounds):
        for s in a.settings:
            env = dict(os.environ)
            for kv in s.split():
                k, v = kv.split("=", 1)
                env[k] = v
            cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--no-cpu-baseline"] + a.bench_args.split()
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
            if p.returncode != 0:
                print(p.stderr[-3000:], file=sys.stderr)
                raise SystemExit(f"bench failed for setting {s!r}")
            line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
            res[s].append({"value": line["value"], "windows": line["repeats"]["values"],
                           "kernel_ms": line["roofline"]["kernel_ms"]})
            print(f"round {r} {s or 'default'}: {line['value']:.0f} {[round(v) for v in line['repeats']['values']]}",
                  flush=True)
    summary = {s or "default": {"median_value": statistics.median(x["value"] for x in v),
                                "runs": v} for s, v in res.items()}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump({"bench_args": a.bench_args, "rounds": a.rounds, "settings": summary}, open(a.out, "w"), indent=1)
    for s, v in summary.items():
        print(f"{s:60s} {v['median_value']:.0f}")


if __name__ == "__main__":
    main()
