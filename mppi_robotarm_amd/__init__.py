"""mppi_robotarm_amd — MI355X-native MPPI rollout-and-reduce engine.

Drop-in for the hot path of junofficial/mppi_RobotArm
(``MPPIControllerForPathTracking.calc_control_input``, control.py:67-152):
the K x T rollout / cost / soft-min / weighted-noise loop runs as a hand-written
HIP kernel for gfx950 behind the C ABI in ``include/mppi_rocm.h``.
"""
from .params import ArmParams, SYS_PARAMS, runpy_config  # noqa: F401

__all__ = ["ArmParams", "SYS_PARAMS", "runpy_config", "MPPIControllerForPathTracking", "RolloutEngine",
           "ChainMPPIController", "ChainEngine", "ChainParams"]


def __getattr__(name):  # lazy: importing the package does not touch the GPU library
    if name == "MPPIControllerForPathTracking":
        from .controller import MPPIControllerForPathTracking
        return MPPIControllerForPathTracking
    if name == "RolloutEngine":
        from .engine import RolloutEngine
        return RolloutEngine
    if name in ("ChainMPPIController", "ChainEngine", "ChainParams"):
        from . import chain
        return getattr(chain, name)
    raise AttributeError(name)
