"""In-tree build of the HIP library for gfx950 (``hipcc`` cross-compiles without a GPU).

Four translation units — ``csrc/mppi_rocm.hip`` (the reference's 2-link arm),
``csrc/mppi_chain.hip`` (the n-link chain of config 5),
``csrc/mppi_npgauss.hip`` (the reference's NumPy noise stream on the device)
and ``csrc/mppi_readback.hip`` (the sampled trajectories' host read-back) —
are compiled in parallel and linked into ``_lib/libmppi_rocm.so``.
"""
from __future__ import annotations

import glob
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SRCS = [os.path.join(CSRC, "mppi_rocm.hip"), os.path.join(CSRC, "mppi_chain.hip"), os.path.join(CSRC, "mppi_npgauss.hip"),
        os.path.join(CSRC, "mppi_readback.hip")]
OUT = os.path.join(HERE, "_lib", "libmppi_rocm.so")
HOST_RNG_SRC = os.path.join(CSRC, "np_legacy_gauss.c")
HOST_RNG_OUT = os.path.join(HERE, "_lib", "libmppi_hostrng.so")
ARCH = os.environ.get("MPPI_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.sep not in cand or os.path.exists(cand)):
            return cand
    return "hipcc"


def build_native(force: bool = False, extra_flags: list[str] | None = None, out: str = OUT) -> str:
    """Compile csrc/*.hip -> _lib/libmppi_rocm.so (skipped when up to date)."""
    deps = SRCS + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(ROOT, "include", "mppi_rocm.h")]
    if not force and os.path.exists(out) and not extra_flags and \
            all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    # host side without contraction: the fp64 host steps (waypoint update, optimal trajectories) fuse only
    # their explicit fma() calls, whatever the CPU target (the chain's target("fma") instance included)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-I", os.path.join(ROOT, "include"),
             "-Xarch_host", "-ffp-contract=off"]
    flags += list(extra_flags or [])
    objs, procs = [], []
    for src in SRCS:
        obj = out + "." + os.path.splitext(os.path.basename(src))[0] + ".o"
        objs.append(obj)
        procs.append(subprocess.Popen([hipcc()] + flags + ["-c", "-o", obj, src]))
    if any(p.wait() != 0 for p in procs):
        raise subprocess.CalledProcessError(1, "hipcc")
    subprocess.run([hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs, check=True)
    for obj in objs:
        os.remove(obj)
    return out


def build_host_rng(force: bool = False) -> str:
    """csrc/np_legacy_gauss.c -> _lib/libmppi_hostrng.so: host C, no contraction, so its values equal NumPy's."""
    deps = (HOST_RNG_SRC, os.path.join(CSRC, "np_glibc_log.h"))
    if not force and os.path.exists(HOST_RNG_OUT) and all(os.path.getmtime(HOST_RNG_OUT) >= os.path.getmtime(d)
                                                          for d in deps):
        return HOST_RNG_OUT
    os.makedirs(os.path.dirname(HOST_RNG_OUT), exist_ok=True)
    subprocess.run(["gcc", "-O3", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math", "-pthread", "-o",
                    HOST_RNG_OUT, HOST_RNG_SRC, "-lm"], check=True)
    return HOST_RNG_OUT


if __name__ == "__main__":
    print(build_native(force=True))
    print(build_host_rng(force=True))
