"""Drop-in latency against the host CPUs the process runs on: the GPU's NUMA node, the CPUs this
process may use, and bench.dropin_latency with the default affinity, then pinned to CPUs of the
GPU's node, then (if allowed) to CPUs of another node.  python tools/numa_lat.py"""
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def cpulist(text):
    out = set()
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


torch.cuda.set_device(0)
allowed = os.sched_getaffinity(0)
bus = torch.cuda.get_device_properties(0).pci_bus_id if hasattr(torch.cuda.get_device_properties(0), "pci_bus_id") else None
print("allowed CPUs:", len(allowed), sorted(allowed)[:8], "...", flush=True)
nodes = {}
for d in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
    nodes[int(d.rsplit("node", 1)[1])] = cpulist(open(os.path.join(d, "cpulist")).read())
print("nodes:", {n: len(c) for n, c in nodes.items()}, "allowed per node:", {n: len(c & allowed) for n, c in nodes.items()})
gpu_nodes = set()
for card in glob.glob("/sys/class/drm/card*/device/numa_node"):
    try:
        gpu_nodes.add(int(open(card).read()))
    except (OSError, ValueError):
        pass
print("GPU numa_node entries visible:", sorted(gpu_nodes), "torch pci bus:", bus, flush=True)


def run(tag):
    med, p90, b2b = bench.dropin_latency(65536, 64, 0)
    print(f"{tag:40s} closed loop {med * 1e3:6.1f} us (p90 {p90 * 1e3:6.1f})  back to back {b2b * 1e3:6.1f} us",
          flush=True)


run("default affinity")
for n, cpus in nodes.items():
    use = cpus & allowed
    if use:
        os.sched_setaffinity(0, use)
        run(f"pinned to node {n} ({len(use)} CPUs)")
os.sched_setaffinity(0, allowed)
run("default affinity again")
