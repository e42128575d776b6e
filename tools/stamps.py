"""Diagnostic timeline of the rollout kernel (stamp build, not the product).

Usage: python tools/stamps.py LIB.so [K T steps]     (WORKLOAD=c5: the 7-link chain engine)
Prints, per recorded step: kernel span, per-workgroup rollout / epilogue
durations, the last workgroup's merge / update, and the sample / partial counts.
"""
import os
import sys

lib = os.path.abspath(sys.argv[1])
os.environ["MPPI_LIB_PATH"] = lib
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mppi_robotarm_amd import _native as N  # noqa: E402
from mppi_robotarm_amd.engine import RolloutEngine  # noqa: E402
from mppi_robotarm_amd.params import ArmParams, X0_RUNPY  # noqa: E402

K = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
T = int(sys.argv[3]) if len(sys.argv) > 3 else 64
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 12
lam = float(os.environ.get("LAMBDA", "100"))
torch.cuda.set_device(0)
path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
if os.environ.get("WORKLOAD") == "c5":   # the 7-link chain engine (config 5)
    from mppi_robotarm_amd.chain import CHAIN7_SIGMA, CHAIN7_X0, ChainEngine, gravity_torque
    eng = ChainEngine(K, T, 0.006, lam, 0.98, CHAIN7_SIGMA, [0.5, 0.5, 5, 5], [5, 5, 50, 50], 0.0, device=0)
    eng.set_step_inputs(CHAIN7_X0, path[:30], np.tile(gravity_torque(CHAIN7_X0[:7]), (T, 1)))
    set_dbg = eng._lib.mppi_chain_debug_set_buffer
    eng.lanes_per_sample = int(os.environ.get("LPS", "1"))
else:
    eng = RolloutEngine(K, T, 0.006, lam, 0.98, np.eye(2) * 20.0, [0.5, 0.5, 5, 5], [5, 5, 50, 50], 0.0, ArmParams(),
                        device=0, lanes_per_sample=int(os.environ.get("LPS", "0")))
    eng.set_step_inputs(X0_RUNPY, path[:30], np.array([[10.0, -2.0]] * T))
    set_dbg = eng._lib.mppi_debug_set_buffer
noise = [eng.philox_noise(1234, i) for i in range(4)]
for i in range(int(os.environ.get("WARM", "0"))):   # converge the device loop first (bench.py's regime)
    eng.rollout(noise[i % 4], fused_update=True)
torch.cuda.synchronize()
dbg = torch.zeros(eng.blocks * 16, dtype=torch.int64, device="cuda")
N.check(set_dbg(eng._ctx, N.C.c_void_p(dbg.data_ptr())), "dbg")
print(f"K={K} T={T} lps={eng.lanes_per_sample} blocks={eng.blocks} lambda={lam} lib={os.path.basename(lib)}")
S_dev = torch.empty(K, dtype=torch.float64, device="cuda")
for i in range(steps):
    dbg.zero_()
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record()
    eng.rollout(noise[i % 4], fused_update=True)
    s1.record()
    torch.cuda.synchronize()
    d = dbg.view(-1, 16).cpu().numpy().astype(np.int64)
    t0 = d[:, 0].min()
    us = lambda v: (v - t0) / 100.0 if v else float("nan")   # slot never written (direct merge: no group level)
    roll = (d[:, 1] - d[:, 0]) / 100.0   # us (100 MHz)
    epi = (d[:, 2] - d[:, 1]) / 100.0
    last = int(np.argmax(d[:, 7]))
    hw = d[:, 8]
    cu = (d[:, 9] & 0xF) * 1000 + ((hw >> 13) & 7) * 100 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 0xF)
    _, per_cu = np.unique(cu, return_counts=True)
    occ = f"blocks/CU {np.bincount(per_cu).tolist()}"
    print(f"step {i:2d}: {occ} | event {s0.elapsed_time(s1)*1e3:6.1f} | rollout med {np.median(roll):5.1f} max {roll.max():5.1f} "
          f"| epi med {np.median(epi):4.1f} max {epi.max():4.1f} | last epi end {us(d[:, 2].max()):5.1f} | final wg: "
          f"grp-arrive {us(d[last, 3]):5.1f} grp-merge {us(d[last, 10]):5.1f} fin-arrive {us(d[last, 4]):5.1f} "
          f"fin-merge {us(d[last, 11]):5.1f} update {us(d[last, 7]):5.1f} | nl med {np.median(d[:, 5]):.0f} max {d[:, 5].max()} "
          f"| rows {d[last, 6]}")
    if d[last, 13] and d[last, 14] and d[last, 13] > d[last, 3]:
        print(f"         merger: rho seen {us(d[last, 13]):5.1f}, weighted rows loaded {us(d[last, 14]):5.1f}")
    if d[:, 15].any():
        print(f"         last rho published {us(d[:, 15].max()):5.1f} (loop end of that wg {us(d[np.argmax(d[:, 15]), 1]):5.1f})"
              f" -> final merge done {us(d[last, 11]):5.1f}")
    gm = d[:, 10][d[:, 10] > 0]
    if len(gm) and (np.arange(len(d)) != last).any():
        others = [b for b in range(len(d)) if b != last and d[b, 10] > 0]
        if others:
            print(f"         level-1 group mergers: {len(others)}, last done {us(max(d[b, 10] for b in others)):5.1f} "
                  f"(final workgroup's update done {us(d[last, 7]):5.1f})")
    st = (d[:, 0] - t0) / 100.0
    late = np.argsort(st)[-3:][::-1]
    print("         start offsets: med %.2f p99 %.2f max %.2f us; latest blocks %s (xcc %s)" % (
        np.median(st), np.percentile(st, 99), st.max(), late.tolist(), (d[late, 9] & 0xF).tolist()))
    if d[:, 12].any():   # loop stamps: prologue, first 4 steps, per-step rate over the second half
        pro = (d[:, 12] - d[:, 0]) / 100.0
        b0 = (d[:, 13] - d[:, 12]) / 100.0
        rate = (d[:, 1] - d[:, 14]) / 100.0 / (T - T // 2) * 1e3
        print(f"         prologue med {np.median(pro):.2f} max {pro.max():.2f} us | first 4 steps med {np.median(b0):.2f} us"
              f" | second-half ns/step med {np.median(rate):.0f} max {rate.max():.0f}")
if os.environ.get("DUMP"):   # the last step: rollout time of the older / younger workgroup sharing a CU
    order = np.argsort(d[:, 0])
    first = {}
    older, younger = [], []
    for b in order:
        if cu[b] in first:
            younger.append(roll[b]); older.append(roll[first[cu[b]]])
        else:
            first[cu[b]] = b
    older, younger = np.array(older), np.array(younger)
    pct = lambda a: " ".join(f"{np.percentile(a, q):6.1f}" for q in (0, 10, 50, 90, 100))
    print(f"rollout pct 0/10/50/90/100: all {pct(roll)}")
    if len(older):
        print(f"  older wg on its CU {pct(older)} | younger {pct(younger)} | start skew med "
              f"{np.median([(d[b, 0] - d[first[cu[b]], 0]) / 100.0 for b in order if first[cu[b]] != b]):.2f} us")
    wid = hw & 0xF
    ob = [first[cu[b]] for b in order if first[cu[b]] != b]
    yb = [b for b in order if first[cu[b]] != b]
    print(f"  HW_ID.WAVE_ID of wave 0: older {np.bincount(wid[ob], minlength=8).tolist()} younger "
          f"{np.bincount(wid[yb], minlength=8).tolist()} | younger blockIdx >= nblocks/2: "
          f"{np.mean(np.array(yb) >= len(d) // 2):.2f}")
    xcc = d[:, 9] & 0xF
    print("  per-XCD median rollout " + " ".join(f"{np.median(roll[xcc == x]):6.1f}" for x in np.unique(xcc)))
u = eng.nominal()
print("final nominal u range", u.min(0), u.max(0))
