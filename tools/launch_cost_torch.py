"""tools/launch_cost.hip's measurements inside a PyTorch process (torch's HIP runtime
initialised first, as under the engine), to compare with the standalone binary."""
import ctypes
import os
import sys

import torch

torch.cuda.init()
torch.empty(1, device="cuda")
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "liblaunch_cost.so"))
sys.stdout.flush()
sys.exit(lib.launch_cost_main())
