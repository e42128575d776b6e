"""The drop-in with run.py's own visualze_sampled_trajs=True at K = 65536, T = 64: wall time of
calc_control_input back to back (device noise, and run.py's exact flags: the default NumPy noise too), and the
read-back of the (K, T, 4) sampled_traj_list by its routes: the fp32 DMA alone (the link floor), the device
widening + fp64 DMA (round 5), and the chunked fp32 DMA widened on host threads (engine.HostReadback) over a
sweep of workers and chunk sizes.  python tools/sampled_latency.py [--quick]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from mppi_robotarm_amd.engine import HostReadback  # noqa: E402

K, T = 65536, 64
quick = "--quick" in sys.argv
torch.cuda.set_device(0)
res = {}
for noise in ("device", "numpy"):
    ms, detail = bench.sampled_latency(K, T, 0, noise=noise)
    res[f"calc_control_input_{noise}_ms"] = ms
    res[f"detail_{noise}"] = detail
    print(f"calc_control_input, sampled trajectories, noise={noise}: median {ms:7.3f} ms  {detail}", flush=True)

tr = torch.randn((K, T, 4), device="cuda", dtype=torch.float32)
torch.cuda.synchronize()


def t(name, fn, n=12):
    v = []
    for _ in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        v.append(time.perf_counter() - t0)
    ms = float(np.median(v[2:])) * 1e3
    res[name] = ms
    print(f"  {name:56s} {ms:7.3f} ms", flush=True)


pin32 = torch.empty((K, T, 4), dtype=torch.float32, pin_memory=True)
pin64 = torch.empty((K, T, 4), dtype=torch.float64, pin_memory=True)
t("fp32 DMA into page-locked (link floor, 67 MB)", lambda: (pin32.copy_(tr), torch.cuda.synchronize()))
t("device widening + fp64 DMA into page-locked (round 5)", lambda: (pin64.copy_(tr.double()), torch.cuda.synchronize()))
dst = np.empty((K, T, 4))
src32 = pin32.numpy()
t("host widening alone, numpy one thread (67 -> 134 MB)", lambda: np.copyto(dst, src32))
configs = [(16, 2 << 20, 2)] if quick else [
    (w, ch, st) for st in (0, 1, 2, 3) for w in (8, 16) for ch in (1 << 20, 2 << 20, 4 << 20)]
for w, ch, st in configs:
    rb = HostReadback(torch.device("cuda", 0), workers=w, chunk=ch, slots=8, streams=st)
    t(f"HostReadback workers={w:2d} chunk={ch * 4 >> 20:2d} MB streams={st}", lambda: rb.run(tr, dst), n=22)
    assert np.array_equal(dst, tr.double().cpu().numpy())
    rb.close()
print(json.dumps(res))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "sampled_latency.json"), "w"), indent=1)
