"""bench.py's drop-in latency legs (closed loop + back to back) repeated, at two call
counts, to see their spread on one box: python tools/lat_compare.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

torch.cuda.set_device(0)
for ticks in (100, 400, 100, 400):
    med, p90, b2b = bench.dropin_latency(65536, 64, 0, ticks=ticks)
    print(f"ticks {ticks:4d}: closed loop {med * 1e3:6.1f} us (p90 {p90 * 1e3:6.1f})  back to back {b2b * 1e3:6.1f} us",
          flush=True)
