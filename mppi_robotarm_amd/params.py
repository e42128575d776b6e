"""Arm and controller parameters of the reference, as plain data.

``SYS_PARAMS`` restates ``sys_params.py:1-13`` (the reference file itself stays
untouched); ``ArmParams`` carries those constants plus the separate link lengths
the cost's kinematics uses (``self.l1 = self.l2 = 1``, control.py:55-56).
``RUNPY_CONFIG`` is the constructor call of ``run.py:25-37``.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def SYS_PARAMS() -> dict:  # noqa: N802 — reference name (sys_params.py:1)
    return {"Ts": 0.0025, "m1": 1, "m2": 1, "l1": 1, "l2": 1, "lc1": 0.5, "lc2": 0.5, "g": 9.81}


@dataclass(frozen=True)
class ArmParams:
    m1: float = 1.0
    m2: float = 1.0
    l1: float = 1.0
    l2: float = 1.0
    lc1: float = 0.5
    lc2: float = 0.5
    g: float = 9.81
    fk_l1: float = 1.0   # control.py:55
    fk_l2: float = 1.0   # control.py:56

    @classmethod
    def from_sys_params(cls, p: dict | None = None, fk_l1: float = 1.0, fk_l2: float = 1.0) -> "ArmParams":
        p = SYS_PARAMS() if p is None else p
        return cls(float(p["m1"]), float(p["m2"]), float(p["l1"]), float(p["l2"]), float(p["lc1"]),
                   float(p["lc2"]), float(p["g"]), float(fk_l1), float(fk_l2))


DT_PLANT = 0.003  # run.py:10
X0_RUNPY = np.array([1.152198236517471885e00, -1.266101672070702344e00, 0.0, 0.0])  # run.py:14-15


def runpy_config() -> dict:
    """Keyword arguments of run.py:25-37 (minus ref_path)."""
    return dict(
        delta_t=DT_PLANT * 2,
        horizon_step_T=30,
        number_of_samples_K=100,
        param_exploration=0.0,
        param_lambda=100.0,
        param_alpha=0.98,
        sigma=np.array([[20.0, 0.0], [0.0, 20.0]]),
        stage_cost_weight=np.array([0.50, 0.50, 5.0, 5.0]),
        terminal_cost_weight=np.array([5.0, 5.0, 50.0, 50.0]),
        visualze_sampled_trajs=True,
    )
