"""Host build of the NumPy-stream helpers (csrc/np_legacy_gauss.c) under AddressSanitizer and UBSan (host code
only; CPU test, kept off the GPU box by .gpurunignore)."""
import os

import pytest

from mppi_robotarm_amd import hostrng


def test_jump_polynomials_clean_under_asan(tmp_path):
    """The jump-polynomial arithmetic (np_legacy_gauss.c reduce_mod / pow_x_mod) under AddressSanitizer and
    UBSan in a host build: no out-of-bounds access of the stack word arrays (the lowest word's terms below bit 33
    once touched a[-1])."""
    import shutil
    import subprocess
    import sys
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("no gcc")
    asan = subprocess.run([gcc, "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    ubsan = subprocess.run([gcc, "-print-file-name=libubsan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(asan) or not os.path.isabs(ubsan):
        pytest.skip("no libasan / libubsan")
    src = os.path.join(os.path.dirname(hostrng.__file__), "csrc", "np_legacy_gauss.c")
    so = tmp_path / "libhostrng_asan.so"
    subprocess.run([gcc, "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-ffp-contract=off", "-pthread", "-shared", "-fPIC", "-o", str(so), src,
                    "-lm"], check=True)
    prog = ("import ctypes as C, numpy as np\n"
            f"lib = C.CDLL({str(so)!r})\n"
            "lib.mppi_np_jump_poly.restype = C.c_int\n"
            "lib.mppi_np_jump_poly.argtypes = [C.c_uint64, C.c_void_p]\n"
            "out = np.zeros(lib.mppi_np_poly_words(), dtype=np.uint64)\n"
            "for J in (624 * 255, 624 * (256 * 5 - 1), 624 * 100000, 12345):\n"
            "    assert lib.mppi_np_jump_poly(J, out.ctypes.data) == 0\n"
            "print('clean')\n")
    env = dict(os.environ, LD_PRELOAD=f"{asan}:{ubsan}", ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([sys.executable, "-c", prog], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "clean" in r.stdout, r.stderr[-2000:]
