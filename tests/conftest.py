import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


def load_paths():
    p = np.load(os.path.join(GOLDEN, "paths.npz"))
    return {"xydq_circle": p["xydq_circle"][:, :4], "trajectory": p["trajectory"],
            "trajectory1": p["trajectory1"]}


STEP_FIXTURES = sorted(os.path.basename(f)[5:-4] for f in glob.glob(os.path.join(GOLDEN, "step_*.npz")))
LOOP_FIXTURES = sorted(os.path.basename(f)[5:-4] for f in glob.glob(os.path.join(GOLDEN, "loop_*.npz")))


def record(kind, **vals):
    """Append one achieved-accuracy record (JSON line) to $MPPI_PARITY_RECORD when
    set: the GPU runs that DESIGN.md's parity tables quote write them there."""
    path = os.environ.get("MPPI_PARITY_RECORD")
    if path:
        import json
        with open(path, "a") as f:
            f.write(json.dumps({"kind": kind, **{k: (float(v) if isinstance(v, (float, np.floating)) else v)
                                                 for k, v in vals.items()}}) + "\n")


def load_step(name):
    return dict(np.load(os.path.join(GOLDEN, f"step_{name}.npz")))


def load_loop(name):
    return dict(np.load(os.path.join(GOLDEN, f"loop_{name}.npz")))


def ctor_kwargs(g):
    return dict(delta_t=float(g["delta_t"]), horizon_step_T=int(g["T"]), number_of_samples_K=int(g["K"]),
                param_exploration=float(g["param_exploration"]), param_lambda=float(g["param_lambda"]),
                param_alpha=float(g["param_alpha"]), sigma=g["sigma"],
                stage_cost_weight=g["stage_cost_weight"], terminal_cost_weight=g["terminal_cost_weight"],
                visualze_sampled_trajs=bool(g["sampled"]))


@pytest.fixture(scope="session")
def paths():
    return load_paths()
