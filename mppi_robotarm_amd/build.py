"""In-tree build of the HIP library for gfx950 (``hipcc`` cross-compiles without a GPU)."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "mppi_rocm.hip")
OUT = os.path.join(HERE, "_lib", "libmppi_rocm.so")
ARCH = os.environ.get("MPPI_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.sep not in cand or os.path.exists(cand)):
            return cand
    return "hipcc"


def build_native(force: bool = False, extra_flags: list[str] | None = None, out: str = OUT) -> str:
    """Compile csrc/mppi_rocm.hip -> _lib/libmppi_rocm.so (skipped when up to date)."""
    deps = [SRC, os.path.join(ROOT, "include", "mppi_rocm.h")]
    if not force and os.path.exists(out) and not extra_flags and \
            all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I", os.path.join(ROOT, "include"), "-o", out, SRC] + list(extra_flags or [])
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    print(build_native(force=True))
