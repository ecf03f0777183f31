"""Static instruction counts per device function of a hipcc -S listing (experiment tooling): VALU,
SALU, LDS, VMEM, scratch and DPP counts, to compare two builds before spending a GPU run."""
import collections
import re
import sys


def stats(path):
    out, fn = collections.OrderedDict(), None
    for line in open(path):
        m = re.match(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$", line)
        if m and not m.group(1).startswith((".L", "$")):
            fn = m.group(1)
            out[fn] = collections.Counter()
            continue
        if fn is None:
            continue
        t = line.strip().split()
        if not t or t[0].startswith((".", ";", "//")) or t[0].endswith(":"):
            continue
        op = t[0]
        c = out[fn]
        c["all"] += 1
        if op.startswith("v_"):
            c["valu"] += 1
            if "dpp" in line or "row_" in line or "quad_perm" in line:
                c["dpp"] += 1
            if "mfma" in op:
                c["mfma"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith("scratch_") or "offen" in line and op.startswith("buffer_"):
            c["scratch"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            c["vmem"] += 1
    return out


if __name__ == "__main__":
    a = stats(sys.argv[1])
    b = stats(sys.argv[2]) if len(sys.argv) > 2 else None
    for fn, c in a.items():
        if c["all"] < 200:
            continue
        line = f"{fn[:40]:40s} " + " ".join(f"{k}={c[k]}" for k in ("all", "valu", "dpp", "salu", "lds", "vmem", "scratch"))
        if b and fn in b:
            d = b[fn]
            line += "  ->  " + " ".join(f"{k}={d[k]}" for k in ("all", "valu", "salu", "lds", "scratch"))
        print(line)
