"""Scratch frames and spill instructions of the step kernel's functions in a hipcc -S listing: the
evidence behind the HBM traffic of the out-of-line substep.  Usage:
    hipcc ... --cuda-device-only -S mmx_kernels.hip -o k.s ; python tools/isa_frame.py k.s [k2.s]
Per function: private segment bytes per lane, VGPRs, scratch stores / loads (the callee-saved save
area and spills), v_writelane / v_readlane (SGPR spills into VGPR lanes and cross-lane reads)."""
import collections
import re
import sys

FUNCS = ("_Z7substepifPf", "mmx_env_step_kernel", "_Z10step_beginRK8MMXStateiPKfii", "_Z11step_finishRK8MMXStatei")


def frames(path):
    txt = open(path).read()
    ops, fn = collections.defaultdict(collections.Counter), None
    for line in txt.split("\n"):
        m = re.match(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$", line)
        if m and not m.group(1).startswith((".L", "$")):
            fn = m.group(1)
            continue
        t = line.strip().split()
        if fn and t:
            for k in ("scratch_store", "scratch_load", "v_writelane", "v_readlane"):
                if t[0].startswith(k):
                    ops[fn][k] += 1
    out = {}
    for f in FUNCS:
        seg = re.search(rf"\.set (?:\.L)?{re.escape(f)}\.private_seg_size, (\d+)(\+max)?", txt)
        vg = re.search(rf"\.set (?:\.L)?{re.escape(f)}\.num_vgpr, (?:max\()?(\d+)", txt)
        out[f] = {"private_seg_bytes_per_lane": int(seg.group(1)) if seg else None,
                  "plus_callees": bool(seg and seg.group(2)), "vgpr": int(vg.group(1)) if vg else None, **ops[f]}
    return out


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(p)
        for f, d in frames(p).items():
            print(f"  {f[:34]:34s} {d}")
