"""A/B timing of two builds of the C ABI in ONE process on the same inputs
(diagnostic tool, not product).  Batches of fused launches alternate between
the builds, so clock and thermal drift hit both alike.

    python tools/ab.py LIB_A.so LIB_B.so [K T batches launches_per_batch]

Prints, per build, the median / min per-launch time (HIP events around each
batch on the launching stream) and B / A.
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mppi_robotarm_amd import _native as N  # noqa: E402
from mppi_robotarm_amd.params import X0_RUNPY, ArmParams  # noqa: E402


def make_ctx(L, K, T, lam, stream):
    a = ArmParams()
    cfg = N.ConfigC()
    cfg.K_local, cfg.T, cfg.K_total, cfg.k_offset = K, T, K, 0
    cfg.delta_t, cfg.param_lambda, cfg.param_alpha, cfg.param_exploration = 0.006, lam, 0.98, 0.0
    cfg.sigma = (C.c_double * 4)(20, 0, 0, 20)
    cfg.stage_cost_weight = (C.c_double * 4)(0.5, 0.5, 5, 5)
    cfg.terminal_cost_weight = (C.c_double * 4)(5, 5, 50, 50)
    cfg.arm = N.ArmParamsC(a.m1, a.m2, a.l1, a.l2, a.lc1, a.lc2, a.g, a.fk_l1, a.fk_l2)
    cfg.lanes_per_sample = int(os.environ.get("LPS", "0"))
    ctx = C.c_void_p()
    rc = L.mppi_ctx_create(C.byref(cfg), 0, C.c_void_p(stream), C.byref(ctx))
    assert rc == 0, L.mppi_last_error()
    return ctx


def main():
    libs = [os.path.abspath(p) for p in sys.argv[1:3]]
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
    T = int(sys.argv[4]) if len(sys.argv) > 4 else 64
    batches = int(sys.argv[5]) if len(sys.argv) > 5 else 40
    per = int(sys.argv[6]) if len(sys.argv) > 6 else 50
    lam = float(os.environ.get("LAMBDA", "100"))
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream().cuda_stream
    path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
    win = np.ascontiguousarray(path[:30])
    u = np.array([[10.0, -2.0]] * T)
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
    runs = []
    for p in libs:
        L = N.open_library(p)
        ctx = make_ctx(L, K, T, lam, stream)
        x0 = np.asarray(X0_RUNPY, dtype=np.float64)
        assert L.mppi_set_step_inputs(ctx, dp(x0), dp(win), 30, dp(u)) == 0
        noise = [torch.empty(T * K * 2, dtype=torch.float32, device="cuda") for _ in range(8)]
        for i, nz in enumerate(noise):
            assert L.mppi_noise_philox(ctx, 1234, i, C.c_void_p(nz.data_ptr())) == 0
        runs.append((L, ctx, noise, []))
    torch.cuda.synchronize()

    def batch(L, ctx, noise, n):
        for i in range(n):
            rc = L.mppi_rollout(ctx, C.c_void_p(noise[i % len(noise)].data_ptr()), None, None, 1)
            assert rc == 0

    for L, ctx, noise, _ in runs:   # warm-up
        batch(L, ctx, noise, 20)
    torch.cuda.synchronize()
    for b in range(batches):
        order = runs if b % 2 == 0 else runs[::-1]
        for L, ctx, noise, times in order:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            batch(L, ctx, noise, per)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3 / per)
    med = []
    for p, (L, ctx, noise, times) in zip(libs, runs):
        t = np.array(times)
        med.append(np.median(t))
        print(f"{os.path.basename(p):36s} median {np.median(t):7.2f} us  min {t.min():7.2f}  max {t.max():7.2f}")
        L.mppi_ctx_destroy(ctx)
    print(f"B/A = {med[1] / med[0]:.4f}  (K={K} T={T} lambda={lam}, {batches} x {per} launches each)")


if __name__ == "__main__":
    main()
