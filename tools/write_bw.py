"""Write-only bandwidth at the noise buffer's size (K = 65536, T = 64: 33.5 MB), to place the
Philox draw (tools/gpu_bm.sh) against the HBM write rate: torch fill_ and hipMemsetAsync."""
import torch

torch.cuda.set_device(0)
n = 65536 * 64 * 2
x = torch.empty(n, dtype=torch.float32, device="cuda")
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for name, fn in (("fill_", lambda: x.fill_(1.0)), ("zero_ (memset)", lambda: x.zero_())):
    for _ in range(20):
        fn()
    ts = []
    for _ in range(50):
        ev[0].record()
        fn()
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
    ts.sort()
    med = ts[len(ts) // 2]
    print(f"{name:16s} median {med:6.2f} us  min {ts[0]:6.2f} us  -> {n * 4 / med / 1e3:7.1f} GB/s")
