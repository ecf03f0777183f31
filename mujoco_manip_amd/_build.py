"""Build libmmx.so (HIP kernels + C-ABI) in-tree for gfx950 with hipcc.

Two variants share the sources: ``libmmx.so`` (the product) and ``libmmx_prof.so``, the same
code compiled with ``-DMMX_PHASE_CLOCK`` so the kernels add per-phase shader-clock cycles into
the stats buffer (selected at load time with ``MMX_PROFILE=1``; never used by the bench).
"""
from __future__ import annotations

import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libmmx.so")
LIB_PROF = os.path.join(PKG, "libmmx_prof.so")
SOURCES = ["mmx_kernels.hip", "mmx_step_l192.hip", "mmx_render.hip", "mmx_png.hip", "mmx_api.cpp"]
HEADERS = ["mmx_kernels.hip", "mmx_model_gen.h", "mmx_render_gen.h", "mmx_state.h", "mmx_device.h", "mmx_geom.h", "mmx_clock.h",
           os.path.join("..", "..", "include", "mmx_api.h"),
           os.path.join("..", "..", "include", "mmx_tuning.h")]
ARCH = os.environ.get("MMX_OFFLOAD_ARCH", "gfx950")
# device-code math: x / y as x * rcp(y) and sqrt without the denormal-scaling wrapper (v_rcp_f32 /
# v_sqrt_f32, <= 1 ulp) instead of the correctly rounded fdiv / sqrt expansions (~10 VALU each).
# The env-step kernel is VALU-issue-bound at 8 envs per CU: -11 % VALU instructions in the substep,
# +3.7 % env steps/s (C3), parity tolerances unchanged.  Host code keeps IEEE semantics.
# r04: no NaN / Inf / signed-zero semantics either (-ffinite-math-only -fno-signed-zeros): selects
# and min / max lose their NaN guards, -2.3 % VALU instructions per env step and +1.1 % env steps/s
# in the interleaved A/B (profiles/archive/r04_ab_finite_math.json), GPU suite unchanged.  The divergence
# detector (NaN / Inf / |v| >= 1e10 -> counted reset) is an integer bit test, exact under any of these.
DEVICE_MATH = ["-Xarch_device", "-freciprocal-math", "-Xarch_device", "-fapprox-func",
               "-Xarch_device", "-ffinite-math-only", "-Xarch_device", "-fno-signed-zeros"]
# gfx950 machine scheduler: the iterative ILP strategy (schedules for latency within the 256-VGPR
# budget the 2-waves-per-SIMD occupancy allows) measured +6.4 % env steps/s over the default
# occupancy-driven scheduler on the C3 bench (max-ilp +2 %, max-memory-clause +0 %).  The option
# is an LLVM backend flag; the host compile accepts and ignores it.
DEVICE_SCHED = ["-mllvm", "-amdgpu-sched-strategy=" + os.environ.get("MMX_SCHED", "iterative-ilp")]
if os.environ.get("MMX_SCHED") == "default":  # experiments: the backend's default scheduler
    DEVICE_SCHED = []
# no SLP vectorisation in device code: at -O3 it packs pairs of independent fp32 ops into
# v_pk_fma_f32 / v_pk_mul_f32 on even-aligned register pairs (2,700 packed ops in the substep); the
# pairing constraints raised the substep's register pressure into scratch spills (frame 480 -> 172 B)
# and the packed ops bought no issue slots: C3 1.905M -> 2.100M env steps/s in the A/B
DEVICE_NOSLP = ["-Xarch_device", "-fno-slp-vectorize"]
# extra compiler flags (experiments only; the committed build uses none)
FLAGS = DEVICE_MATH + DEVICE_SCHED + DEVICE_NOSLP + os.environ.get("MMX_EXTRA_FLAGS", "").split()
# per-source flags.  The env-step kernel (r04 end): floating-point reassociation in device code
# (-fassociative-math; explicit fmaf / DPP / readlane reductions keep their written order), -2 %
# VALU instructions per env step, C3 +0.9 % in the interleaved A/B (profiles/archive/r04_ab_assoc.json),
# GPU suite unchanged.  Not the renderer, whose shared-edge functions rely on one evaluation order.
SOURCE_FLAGS = {"mmx_kernels.hip": ["-Xarch_device", "-fassociative-math"],
                "mmx_step_l192.hip": ["-Xarch_device", "-fassociative-math"]}


# test-only builds of the step kernel (tests/test_overflow_kat.py): the same sources with a define that
# forces a rare path; linked with the product objects of the other sources
TEST_VARIANTS = {
    # a 4-entry collision candidate list (product: 320): the sphere-test overflow path, flagged as
    # ERR_CON_OVERFLOW in env_error
    "libmmx_col4.so": ["MMX_COL_LIST=4", "MMX_CAND_CAP=4"],
    # a 1-entry persistent broadphase list: every collision pass runs the full 780-pair prune (the
    # list-vs-full-prune bit-identity test)
    "libmmx_nolist.so": ["MMX_CAND_CAP=1"],
}


def lib_path(profile: bool = False) -> str:
    return LIB_PROF if profile else LIB


def _stale(lib: str) -> bool:
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _compile(src: str, profile: bool, verbose: bool) -> str:
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    obj = os.path.join(CSRC, os.path.splitext(src)[0] + ("_prof" if profile else "") + ".o")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", os.path.join(CSRC, src), "-o", obj]
    cmd[1:1] = FLAGS + SOURCE_FLAGS.get(src, [])
    if profile:
        cmd.insert(1, "-DMMX_PHASE_CLOCK=1")
        cmd.insert(1, f"-DMMX_PROBE={int(os.environ.get('MMX_PROBE', '1'))}")
    if src.endswith(".cpp"):
        cmd.insert(1, "-xhip")
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    return obj


def _compile_test_variant(name: str, verbose: bool) -> str:
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    obj = os.path.join(CSRC, "mmx_kernels_" + os.path.splitext(name)[0] + ".o")
    cmd = [hipcc] + FLAGS + SOURCE_FLAGS["mmx_kernels.hip"] + [f"-D{d}" for d in TEST_VARIANTS[name]] + [
        f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", os.path.join(CSRC, "mmx_kernels.hip"), "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    return obj


def build(force: bool = False, verbose: bool = False, profile: bool | None = False) -> str:
    """Build one variant (profile=False/True) or both (profile=None, which also builds the test-only
    TEST_VARIANTS); returns the product path."""
    variants = [False, True] if profile is None else [profile]
    variants = [v for v in variants if force or _stale(lib_path(v))]
    tests = [n for n in TEST_VARIANTS if profile is None and (force or _stale(os.path.join(PKG, n)))]
    if variants or tests:
        jobs = [(src, v) for v in variants for src in SOURCES]
        with ThreadPoolExecutor(max_workers=len(jobs) + len(tests)) as ex:
            tobjs = [ex.submit(_compile_test_variant, n, verbose) for n in tests]
            objs = list(ex.map(lambda j: _compile(j[0], j[1], verbose), jobs))
            tobjs = [f.result() for f in tobjs]
        hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
        for v in variants:
            mine = [o for o, (_, vv) in zip(objs, jobs) if vv == v]
            subprocess.check_call([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib_path(v)] + mine)
        for n, kobj in zip(tests, tobjs):  # the product's objects of the other sources
            rest = [os.path.join(CSRC, os.path.splitext(src)[0] + ".o") for src in SOURCES if src != "mmx_kernels.hip"]
            subprocess.check_call([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", os.path.join(PKG, n), kobj] + rest)
    return lib_path(bool(profile))


if __name__ == "__main__":
    print(build(force=True, verbose=True, profile=None))


def build_variant(out: str, defines: list[str], profile: bool = True) -> str:
    """Diagnostic / experiment build of the same sources with extra -D defines into `out`
    (e.g. build/libmmx_prof5.so for probe set 5); loaded with MMX_LIB_PATH.  Not the product."""
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tag = os.path.splitext(os.path.basename(out))[0]
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)

    def one(src):
        obj = os.path.join(os.path.dirname(os.path.abspath(out)), f"{tag}_{os.path.splitext(src)[0]}.o")
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", os.path.join(CSRC, src), "-o", obj]
        cmd[1:1] = FLAGS + SOURCE_FLAGS.get(src, []) + [f"-D{d}" for d in defines] + (["-DMMX_PHASE_CLOCK=1"] if profile else [])
        if src.endswith(".cpp"):
            cmd.insert(1, "-xhip")
        subprocess.check_call(cmd)
        return obj

    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(one, SOURCES))
    subprocess.check_call([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs)
    return out
