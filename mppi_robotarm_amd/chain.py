"""n-link planar chain MPPI (BASELINE config 5: 7-DoF, K=131072 T=128).

The reference has no 7-DoF model; this model is build-defined (equations in
``oracle/chain_oracle.py`` and ``include/mppi_rocm.h``) and reduces to the
reference ``_F`` (control.py:234-263) at n = 2 with inertia := link length.
``ChainMPPIController`` keeps the reference controller's interface
(control.py:21-152) with ``dim_u = n``, ``dim_x = 2n``:
``calc_control_input(observed_x)`` -> (u0, u_seq, optimal_traj (T, 2n),
sampled_traj_list (K, T, 2n)); the cost is control.py:174-232 on the end
effector (x, y) and the first two joint rates (xydq_circle.txt's columns).

Device work runs in ``csrc/mppi_chain.hip`` through ``mppi_chain_*``; the host
keeps the O(T n) work in fp64 (nearest-waypoint update, noise draw, median
filter, update, shift), as ``controller.py`` does for the 2-link arm.
"""
from __future__ import annotations

import ctypes as C
import weakref
from dataclasses import dataclass, field

import numpy as np
import torch
from scipy.ndimage import median_filter

from . import _native as N
from . import hostrng
from .controller import SampledReadback, _noise_check, _pinned_zbuf, first_min_index
from .distributed import attach_exchange, check_exchange, exchange_partials, same_on_all_ranks, shard_geometry

SEARCH_IDX_LEN = 30  # control.py:203


def _tup(v):
    return field(default_factory=lambda: tuple(v))


@dataclass(frozen=True)
class ChainParams:
    """Link constants of the chain ("extended sys_params.py").  Defaults: the
    config-5 arm — 7 uniform slender links of 1 kg, total reach 2 m (the 2-link
    arm's l1 + l2), centre of mass at mid-link, I = m l^2 / 12, and joint drives
    with 0.1 kg m^2 armature and 1 N m s / rad viscous damping (without them the
    undamped 7-link chain collapses from its gravity-held pose and a few percent
    of T = 128 rollouts overflow)."""
    m: tuple = _tup([1.0] * 7)
    l: tuple = _tup([2.0 / 7.0] * 7)
    lc: tuple = _tup([1.0 / 7.0] * 7)
    I: tuple = _tup([(2.0 / 7.0) ** 2 / 12.0] * 7)
    fk: tuple = _tup([2.0 / 7.0] * 7)
    J: tuple = _tup([0.1] * 7)
    b: tuple = _tup([1.0] * 7)
    g: float = 9.81

    @property
    def n(self) -> int:
        return len(self.m)

    @staticmethod
    def from_arm2(arm=None) -> "ChainParams":
        """The reference 2-link model (control.py:11-18, 241-245): inertia := link length."""
        from .params import ArmParams
        a = ArmParams() if arm is None else arm
        return ChainParams(m=(a.m1, a.m2), l=(a.l1, a.l2), lc=(a.lc1, a.lc2), I=(a.l1, a.l2),
                           fk=(a.fk_l1, a.fk_l2), J=(0.0, 0.0), b=(0.0, 0.0), g=a.g)


# Config-5 start pose: the end effector on xydq_circle.txt's first waypoint
# (least-squares IK with a smooth bend, computed once), at rest.
CHAIN7_X0 = np.array([1.481492] + [-0.320757] * 6 + [0.0] * 7)
# Noise covariance scaled with the gravity load each joint carries.
CHAIN7_SIGMA = np.diag([20.0, 16.0, 12.0, 8.0, 4.0, 2.0, 1.0])


def gravity_torque(q, P: ChainParams = ChainParams()) -> np.ndarray:
    """Joint torques that hold the chain still at q (the nominal's natural start)."""
    m, l, lc = map(np.asarray, (P.m, P.l, P.lc))
    tail = np.array([m[k + 1:].sum() for k in range(P.n)])
    g_th = P.g * (m * lc + l * tail) * np.cos(np.cumsum(q))
    return np.cumsum(g_th[::-1])[::-1]


def chain7_config() -> dict:
    """Constructor kwargs of the config-5 controller: run.py's constants (run.py:25-37) with the 7-link Sigma."""
    return dict(delta_t=0.006, horizon_step_T=128, number_of_samples_K=131072, param_exploration=0.0,
                param_lambda=100.0, param_alpha=0.98, sigma=CHAIN7_SIGMA.copy(),
                stage_cost_weight=np.array([0.5, 0.5, 5.0, 5.0]),
                terminal_cost_weight=np.array([5.0, 5.0, 50.0, 50.0]))


def _raw_stream(index: int) -> int:
    """Handle of torch's current stream on device `index` without building a Stream object."""
    get = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    return get(index) if get is not None else torch.cuda.current_stream(index).cuda_stream


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class ChainEngine:
    """Owns one ``mppi_chain_ctx`` (one device, one shard of samples); noise layout [T][K_local][n] fp32."""

    def __init__(self, K_local: int, T: int, delta_t: float, param_lambda: float, param_alpha: float, sigma,
                 stage_cost_weight, terminal_cost_weight, param_exploration: float = 0.0,
                 chain: ChainParams = ChainParams(), K_total: int | None = None, k_offset: int = 0,
                 device: int | torch.device | None = None, precision: str = "f32", lanes_per_sample: int = 0,
                 param_gamma: float | None = None):
        self._lib = N.load()
        if precision not in ("f32", "f64"):
            raise ValueError("precision must be 'f32' or 'f64'")
        self.precision = precision
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", device if isinstance(device, int) else device.index)
        self.n = chain.n
        self.K_local, self.T = int(K_local), int(T)
        self.K_total = int(K_total if K_total is not None else K_local)
        self.k_offset = int(k_offset)
        cfg = N.ChainConfigC()
        cfg.K_local, cfg.T, cfg.K_total, cfg.k_offset = self.K_local, self.T, self.K_total, self.k_offset
        cfg.delta_t, cfg.param_lambda = float(delta_t), float(param_lambda)
        cfg.param_alpha, cfg.param_exploration = float(param_alpha), float(param_exploration)
        sig = np.asarray(sigma, dtype=np.float64)
        if sig.shape != (self.n, self.n):
            raise ValueError(f"sigma must be {self.n} x {self.n}")
        for i, v in enumerate(sig.ravel()):
            cfg.sigma[i] = float(v)
        for i in range(4):
            cfg.stage_cost_weight[i] = float(stage_cost_weight[i])
            cfg.terminal_cost_weight[i] = float(terminal_cost_weight[i])
        cfg.chain.n = self.n
        for f in ("m", "l", "lc", "I", "fk", "J", "b"):
            arr = getattr(cfg.chain, f)
            for i, v in enumerate(getattr(chain, f)):
                arr[i] = float(v)
        cfg.chain.g = float(chain.g)
        cfg.precision = 1 if precision == "f64" else 0
        cfg.lanes_per_sample = int(lanes_per_sample)
        # gamma as given (control.py:45 fixes it at construction); None: lambda (1 - alpha)
        cfg.param_gamma = float("nan") if param_gamma is None else float(param_gamma)
        with torch.cuda.device(self.device):
            self.stream = torch.cuda.current_stream(self.device)
            ctx = C.c_void_p()
            N.check(self._lib.mppi_chain_ctx_create(C.byref(cfg), self.device.index,
                                                    C.c_void_p(self.stream.cuda_stream), C.byref(ctx)),
                    "mppi_chain_ctx_create")
        self._ctx = ctx
        blocks, threads, poll, lps = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        N.check(self._lib.mppi_chain_ctx_info(ctx, C.byref(blocks), C.byref(threads), C.byref(poll), C.byref(lps)),
                "mppi_chain_ctx_info")
        self.blocks, self.threads, self.lanes_per_sample = blocks.value, threads.value, lps.value
        self.handoff = "poll" if poll.value else "counter"
        self.partial_len = 2 + self.n * self.T

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            self._lib.mppi_chain_ctx_destroy(self._ctx)
            self._ctx = None
        self._noise_stage = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def _sync_stream(self):
        """Follow torch's current stream; the new stream first waits for the old one."""
        if _raw_stream(self.device.index) == self.stream.cuda_stream:   # the usual case, ~0.3 us
            return
        s = torch.cuda.current_stream(self.device)
        if s.cuda_stream != self.stream.cuda_stream:
            s.wait_stream(self.stream)
            self.stream = s
            N.check(self._lib.mppi_chain_set_stream(self._ctx, C.c_void_p(s.cuda_stream)), "mppi_chain_set_stream")

    def new_noise(self) -> torch.Tensor:
        return torch.empty((self.T, self.K_local, self.n), dtype=torch.float32, device=self.device)

    def new_partial(self) -> torch.Tensor:
        return torch.empty(self.partial_len, dtype=torch.float64, device=self.device)

    def upload_noise(self, eps_ktn: np.ndarray, out: torch.Tensor | None = None) -> torch.Tensor:
        """Reference-order noise (K_local, T, n) -> device [T][K_local][n] fp32."""
        out = self.new_noise() if out is None else out
        # the fp64 draw as it is (one pageable copy, the host array free once it returns), then the transpose
        # and the fp64 -> fp32 rounding (to nearest, as NumPy's astype) in one device copy: the host transpose,
        # conversion and per-call page-locked buffer cost ~70 ms at K = 65536, T = 64
        eps = np.ascontiguousarray(eps_ktn, dtype=np.float64)
        stage = getattr(self, "_noise_stage", None)
        if stage is None or tuple(stage.shape) != eps.shape:
            stage = self._noise_stage = torch.empty(eps.shape, dtype=torch.float64, device=self.device)
        stage.copy_(torch.from_numpy(eps))
        out.copy_(stage.permute(1, 0, 2))
        return out

    def upload_std_noise(self, noise, z: torch.Tensor, out: torch.Tensor) -> torch.Event:
        """As RolloutEngine.upload_std_noise, into the chain's [T][K_local][n] layout."""
        from .engine import _upload_std
        return _upload_std(self, noise, z, out, (1, 0, 2))

    def set_step_inputs(self, x0, window, u=None) -> None:
        self._sync_stream()
        x0 = np.ascontiguousarray(np.asarray(x0, dtype=np.float64).ravel()[:2 * self.n])
        win = np.ascontiguousarray(np.asarray(window, dtype=np.float64)[:, :4])
        if win.ndim != 2 or win.shape[0] < 1 or win.shape[0] > N.MPPI_SEARCH_LEN:
            raise ValueError("window must have 1..30 rows of [x, y, dq1, dq2]")
        uu = None if u is None else np.ascontiguousarray(np.asarray(u, dtype=np.float64).reshape(self.T, self.n))
        N.check(self._lib.mppi_chain_set_step_inputs(self._ctx, _dptr(x0), _dptr(win), win.shape[0],
                                                     _dptr(uu) if uu is not None else None),
                "mppi_chain_set_step_inputs")
        self._keep = (x0, win, uu)

    def exchange_handle(self, world: int) -> bytes:
        """Allocate this rank's exchange inbox for `world` ranks; its IPC handle (64 B)."""
        buf = C.create_string_buffer(N.MPPI_IPC_HANDLE_BYTES)
        N.check(self._lib.mppi_chain_exchange_handle(self._ctx, int(world), buf), "mppi_chain_exchange_handle")
        return buf.raw

    def exchange_attach(self, rank: int, world: int, handles) -> None:
        """Map every rank's inbox (handles in rank order); then rollout(..., exchange=True)."""
        blob = b"".join(bytes(h) for h in handles)
        if len(blob) != world * N.MPPI_IPC_HANDLE_BYTES:
            raise ValueError("one 64-byte handle per rank")
        N.check(self._lib.mppi_chain_exchange_attach(self._ctx, int(rank), int(world),
                                                     C.create_string_buffer(blob, len(blob))),
                "mppi_chain_exchange_attach")
        self.exchange_world = int(world)

    def rollout(self, noise: torch.Tensor, S_out: torch.Tensor | None = None,
                partial_out: torch.Tensor | None = None, fused_update: bool = False, exchange: bool = False,
                host_out: bool = False) -> None:
        self._sync_stream()
        self._check_noise(noise)
        if S_out is not None:
            assert S_out.dtype == torch.float64 and S_out.numel() >= self.K_local and S_out.device == self.device
        if partial_out is not None:
            assert partial_out.dtype == torch.float64 and partial_out.numel() >= self.partial_len
        N.check(self._lib.mppi_chain_rollout(self._ctx, C.c_void_p(noise.data_ptr()),
                                             C.c_void_p(S_out.data_ptr()) if S_out is not None else None,
                                             C.c_void_p(partial_out.data_ptr()) if partial_out is not None else None,
                                             (N.MPPI_FLAG_FUSED_UPDATE if fused_update else 0)
                                             | (N.MPPI_FLAG_EXCHANGE if exchange else 0)
                                             | (N.MPPI_FLAG_HOST_OUT if host_out else 0)),
                "mppi_chain_rollout")

    def merge(self, partials: torch.Tensor, n: int, fused_update: bool = False) -> None:
        self._sync_stream()
        assert partials.dtype == torch.float64 and partials.is_contiguous()
        assert partials.numel() >= n * self.partial_len
        N.check(self._lib.mppi_chain_merge_partials(self._ctx, C.c_void_p(partials.data_ptr()), int(n),
                                                    N.MPPI_FLAG_FUSED_UPDATE if fused_update else 0),
                "mppi_chain_merge_partials")

    def weighted_noise(self) -> np.ndarray:
        self._sync_stream()
        out = np.zeros((self.T, self.n))
        N.check(self._lib.mppi_chain_get_weighted_noise(self._ctx, _dptr(out)), "mppi_chain_get_weighted_noise")
        return out

    def nominal(self) -> np.ndarray:
        self._sync_stream()
        out = np.zeros((self.T, self.n))
        N.check(self._lib.mppi_chain_get_nominal(self._ctx, _dptr(out)), "mppi_chain_get_nominal")
        return out

    def wait_outputs(self, x0=None) -> tuple[np.ndarray, np.ndarray | None]:
        """After rollout(..., fused_update=True): the shifted nominal (T, n) and, with x0 (2n,), the fp64
        optimal trajectory (T, 2n) of the update before its shift (mppi_chain_wait_outputs)."""
        self._sync_stream()
        u = np.empty((self.T, self.n))
        traj = None
        xp = None
        if x0 is not None:
            traj = np.empty((self.T, 2 * self.n))
            xv = np.ascontiguousarray(np.asarray(x0, dtype=np.float64).ravel()[:2 * self.n])
            xp = _dptr(xv)
        N.check(self._lib.mppi_chain_wait_outputs(self._ctx, xp, _dptr(u), _dptr(traj) if traj is not None else None),
                "mppi_chain_wait_outputs")
        return u, traj

    def last_eta(self) -> float:
        """eta = sum_k exp(-(S_k - min S) / lambda) of the last update (wait_outputs) or weighted noise
        (weighted_noise) read back: 1 for one-hot weights, eta - 1 the weight outside the best sample."""
        v = C.c_double()
        N.check(self._lib.mppi_chain_last_eta(self._ctx, C.byref(v)), "mppi_chain_last_eta")
        return v.value

    def optimal_traj_host(self, x0, u_new) -> np.ndarray:
        """(T, 2n) fp64 optimal trajectory of control.py:129-134 from the updated, not yet shifted
        controls u_new (T, n), on the host (mppi_chain_optimal_traj_host)."""
        xv = np.ascontiguousarray(np.asarray(x0, dtype=np.float64).ravel()[:2 * self.n])
        uv = np.ascontiguousarray(np.asarray(u_new, dtype=np.float64).reshape(self.T, self.n))
        out = np.empty((self.T, 2 * self.n))
        N.check(self._lib.mppi_chain_optimal_traj_host(self._ctx, _dptr(xv), _dptr(uv), _dptr(out)),
                "mppi_chain_optimal_traj_host")
        return out

    def trajectories(self, base_u=None, noise: torch.Tensor | None = None, K: int | None = None) -> torch.Tensor:
        """(K, T, 2n) fp32 states of the off-by-one re-roll (control.py:129-145 analogue)."""
        self._sync_stream()
        K = self.K_local if K is None else int(K)
        out = torch.empty((K, self.T, 2 * self.n), dtype=torch.float32, device=self.device)
        bu = None if base_u is None else np.ascontiguousarray(np.asarray(base_u, dtype=np.float64).reshape(
            self.T, self.n))
        if noise is not None:
            self._check_noise(noise)
        N.check(self._lib.mppi_chain_rollout_traj(self._ctx, _dptr(bu) if bu is not None else None,
                                                  C.c_void_p(noise.data_ptr()) if noise is not None else None,
                                                  K, C.c_void_p(out.data_ptr())),
                "mppi_chain_rollout_traj")
        self._keep_traj = bu
        return out

    def debug_slots(self, noise: torch.Tensor, S_out: torch.Tensor | None = None) -> np.ndarray:
        """Tests: one rollout (as rollout(noise, S_out)) through the slot-recording build of the
        kernel -> the window slot every sample picked at every step, (K_local, T) int32
        (mppi_chain_debug_slots; the 7-link chain only)."""
        self._sync_stream()
        self._check_noise(noise)
        if S_out is not None:
            assert S_out.dtype == torch.float64 and S_out.numel() >= self.K_local and S_out.device == self.device
        slots = torch.full((self.K_local, self.T), -1, dtype=torch.int32, device=self.device)
        N.check(self._lib.mppi_chain_debug_slots(self._ctx, C.c_void_p(noise.data_ptr()),
                                                 C.c_void_p(S_out.data_ptr()) if S_out is not None else None,
                                                 C.c_void_p(slots.data_ptr())), "mppi_chain_debug_slots")
        return slots.cpu().numpy()

    def philox_noise(self, seed: int, step: int = 0, out: torch.Tensor | None = None) -> torch.Tensor:
        self._sync_stream()
        out = self.new_noise() if out is None else out
        self._check_noise(out)
        N.check(self._lib.mppi_chain_noise_philox(self._ctx, int(seed) & (2 ** 64 - 1), int(step) & (2 ** 64 - 1),
                                                  C.c_void_p(out.data_ptr())), "mppi_chain_noise_philox")
        return out

    def synchronize(self) -> None:
        N.check(self._lib.mppi_chain_sync(self._ctx), "mppi_chain_sync")

    def _check_noise(self, noise: torch.Tensor) -> None:
        shape = (self.T, self.K_local, self.n)
        if (noise.dtype != torch.float32 or not noise.is_contiguous() or noise.device != self.device
                or tuple(noise.shape) != shape):
            raise ValueError(f"noise must be a contiguous fp32 {shape} tensor on {self.device}")


class ChainMPPIController:
    """control.py:20-152 for the n-link chain (dim_u = n, dim_x = 2n).

    ``precision``: the rollout arithmetic.  "f32" (fastest) or "f64" (ChainStateD, ~2.9x the time), or "auto"
    (the default): fp32 while the weights are one-hot, fp64 where they spread.  In fp32 a nearest-waypoint tie
    of a weighted sample can move its S by a whole stage-cost step, which reaches w_eps only when
    more than one sample carries weight; so after each fp32 step the spread of its weights, eta - 1 =
    sum_k exp(-(S_k - min S) / lambda) - 1 (mppi_chain_last_eta), is checked, and a step whose weights spread
    (eta - 1 > ETA_TOL) is run again in fp64 from the same inputs, as are the steps after it until the weights
    are one-hot again.  run.py's lambda = 100 keeps them one-hot (eta - 1 ~ 0): the fp32 step alone."""

    ETA_TOL = 1e-6   # weight outside the best sample above which precision="auto" takes the fp64 rollout

    def __init__(self, delta_t: float = 0.006, ref_path=0, horizon_step_T: int = 128,
                 number_of_samples_K: int = 131072, param_exploration: float = 0.0, param_lambda: float = 100.0,
                 param_alpha: float = 0.98, sigma: np.ndarray = CHAIN7_SIGMA,
                 stage_cost_weight: np.ndarray = np.array([0.5, 0.5, 5.0, 5.0]),
                 terminal_cost_weight: np.ndarray = np.array([5.0, 5.0, 50.0, 50.0]),
                 visualize_optimal_traj=True, visualze_sampled_trajs=False, *, chain: ChainParams = ChainParams(),
                 u_init=None, device: int | None = None, verbose: bool = False, noise: str = "numpy", seed: int = 0,
                 process_group=None, exchange: str = "auto", precision: str = "auto",
                 numpy_noise_on_device: bool = True) -> None:
        self.chain = chain
        if precision not in ("auto", "f32", "f64"):
            raise ValueError("precision must be 'auto', 'f32' or 'f64'")
        self.precision = precision
        self.dim_u, self.dim_x = chain.n, 2 * chain.n
        self.T, self.K = horizon_step_T, number_of_samples_K
        self.param_exploration, self.param_lambda, self.param_alpha = param_exploration, param_lambda, param_alpha
        self.param_gamma = self.param_lambda * (1.0 - self.param_alpha)
        self.Sigma = np.asarray(sigma, dtype=np.float64)
        self.stage_cost_weight, self.terminal_cost_weight = stage_cost_weight, terminal_cost_weight
        self.visualize_optimal_traj, self.visualze_sampled_trajs = visualize_optimal_traj, visualze_sampled_trajs
        self.delta_t, self.ref_path = delta_t, ref_path
        u0 = np.zeros(self.dim_u) if u_init is None else np.asarray(u_init, dtype=np.float64)
        self.u_prev = np.tile(u0, (self.T, 1)) if u0.ndim == 1 else u0.astype(np.float64).copy()
        self.prev_waypoints_idx = 0
        if noise not in ("numpy", "device"):
            raise ValueError("noise must be 'numpy' or 'device'")
        self.verbose, self.noise_source, self.seed = verbose, noise, int(seed)
        self.process_group = process_group
        if exchange not in ("auto", "launch", "rccl"):
            raise ValueError("exchange must be 'auto', 'launch' or 'rccl'")
        self.exchange = exchange      # multi-GPU: as MPPIControllerForPathTracking
        self._device = device
        self._slots = {}               # rollout precision -> the parked state of its engine (_SLOT fields)
        self._active = None            # the precision whose engine the fields below hold
        self._engine = None
        self._engine_built_for = None
        self._xmode = None
        self._noise_ready = None       # (seed, step) of the device noise already in the buffer
        self._spread = False           # precision="auto": the last step's weights were spread (next step fp64)
        self._x_failed = False         # an in-launch exchange failed (a late rank): the all-gather from then on
        self.last_precision = None     # the rollout precision of the last step's result
        self.last_eta = None           # and the spread of its weights (eta, mppi_chain_last_eta)
        self._last_sampled = None      # the previous call's sampled_traj_list (_fresh_sampled)
        self._sampled_pool = SampledReadback()   # sampled_traj_list's read-back buffers
        self._step_count = 0
        self.keep_costs = False
        self.last_S = None
        self.numpy_noise_on_device = numpy_noise_on_device   # noise="numpy": the same stream drawn on the device
        self._npdev = None             # its engine.NpDeviceStream (False: unavailable here)
        self._npre = None              # (start state, spec, buffer) of the next call's draw, queued beside a step
        self._np_spec = None           # (spec, plan) of this call's device draw
        self._np_left = None           # the state it left np.random in
        self._np_plan = None           # (Sigma bytes, dtype, hostrng.device_plan) of the last draw
        self._npre_used = 0            # calls that used the queued draw
        self._np_recorded = {}         # id -> weakref of the noise buffers already record_stream'ed on the draw stream
        self._np_stream = None         # the stream of the queued draws
        self._np_ev = None

    # the per-engine fields: the active engine's live here, the others' are parked in _slots
    _SLOT = ("_engine", "_engine_built_for", "_xmode", "_noise_ready", "_noise_dev", "_noise_alt", "_partial",
             "_S_dev", "_gathered")

    def _activate(self, precision: str) -> None:
        """Make the engine of `precision` (built on first use) the one the fields above refer to."""
        if self._active == precision:
            return
        if self._active is not None:
            self._slots[self._active] = {f: getattr(self, f, None) for f in self._SLOT}
        parked = self._slots.pop(precision, {})
        for f in self._SLOT:
            setattr(self, f, parked.get(f))
        self._active = precision

    def _shard(self):
        if self.process_group is None:
            return 1, 0
        import torch.distributed as dist
        return dist.get_world_size(self.process_group), dist.get_rank(self.process_group)

    def _engine_key(self):
        """What the engine bakes in that a call reads (as MPPIControllerForPathTracking._engine_key:
        K, T, Sigma, lambda, gamma, the cost weights, the exploration split, delta_t, the chain and
        the rollout precision); a change rebuilds the engine before the next step."""
        return (int(self.K), int(self.T), np.asarray(self.Sigma, dtype=np.float64).tobytes(), float(self.param_lambda),
                float(self.param_gamma), np.asarray(self.stage_cost_weight, dtype=np.float64).tobytes(),
                np.asarray(self.terminal_cost_weight, dtype=np.float64).tobytes(), float(self.param_exploration),
                float(self.delta_t), self.chain, self._active)

    def _get_engine(self, key=None) -> ChainEngine:
        key = self._engine_key() if key is None else key
        if self._engine is not None and key != self._engine_built_for:
            self._close_active()
        if self._engine is None:
            world, rank = self._shard()
            K_local, k_offset = shard_geometry(self.K, world, rank)
            device = self._device if self._device is not None else torch.cuda.current_device()
            # gamma is fixed at construction in the reference (control.py:45) while lambda is
            # re-read per call: the engine takes gamma as given, as the 2-link engine does
            self._engine = ChainEngine(K_local, self.T, self.delta_t, self.param_lambda, self.param_alpha, self.Sigma,
                                       self.stage_cost_weight, self.terminal_cost_weight, self.param_exploration,
                                       self.chain, K_total=self.K, k_offset=k_offset, device=device,
                                       precision=self._active, param_gamma=self.param_gamma)
            self._noise_dev = self._engine.new_noise()
            self._noise_alt = None                         # the queued draw's buffer, made on first use
            self._partial = self._engine.new_partial()
            self._S_dev = torch.empty(K_local, dtype=torch.float64, device=self._engine.device)
            if world > 1:
                self._gathered = torch.empty(world * self._engine.partial_len, dtype=torch.float64,
                                             device=self._engine.device)
            self._xmode = None
            self._engine_built_for = key
        return self._engine

    def _multi_setup(self, eng: ChainEngine, noise_check) -> None:
        """As MPPIControllerForPathTracking._multi_setup: the ranks agree on the noise
        stream; the in-launch exchange if its self-check passes, else RCCL."""
        pg = self.process_group
        if not same_on_all_ranks((self.K, self.T, self.noise_source, self.seed, noise_check), pg):
            raise RuntimeError("ranks disagree on the noise stream: every rank must seed np.random identically "
                               "(and pass the same seed / K / T)")
        mode = "rccl"
        if self.exchange != "rccl" and not self._x_failed:   # after a failed exchange: the all-gather for good
            self.exchange_report = {}                      # why an exchange was (not) picked (distributed.py)
            ok = attach_exchange(eng, pg, report=self.exchange_report)
            ok = ok and check_exchange(eng, self._noise_dev, self._partial, self._gathered, pg,
                                       report=self.exchange_report)
            if not ok and self.exchange == "launch":
                raise RuntimeError("the in-launch exchange failed its self-check (exchange='launch')")
            mode = "launch" if ok else "rccl"
        self._xmode = mode

    def _effector(self, q):
        th = np.cumsum(q)
        fk = np.asarray(self.chain.fk)
        return float((fk * np.cos(th)).sum()), float((fk * np.sin(th)).sum())

    def _get_nearest_waypoint(self, x: float, y: float, update_prev_idx: bool = False):
        """control.py:200-232 on the end-effector position, host fp64"""
        prev_idx = self.prev_waypoints_idx
        win = self.ref_path[prev_idx:(prev_idx + SEARCH_IDX_LEN)]
        nearest_idx = first_min_index(((x - win[:, 0]) ** 2 + (y - win[:, 1]) ** 2) * 100) + prev_idx
        if update_prev_idx:
            if self.verbose:
                print(f"0     prev_idx = {prev_idx}")
                print(f"0     nearest_idx = {nearest_idx}")
                print("======================updated=======================")
            self.prev_waypoints_idx = nearest_idx
        return nearest_idx

    def _custom_epsilon(self) -> bool:
        """_calc_epsilon replaced on the instance or a subclass: the caller's noise, not the reference's draw."""
        return "_calc_epsilon" in self.__dict__ or type(self)._calc_epsilon is not ChainMPPIController._calc_epsilon

    def _reference_noise(self):
        """control.py:84 as MPPIControllerForPathTracking._reference_noise: the standard normals into a
        page-locked buffer and the transform on the device when Sigma allows it (the chain's diagonal Sigma
        does), else _calc_epsilon's array."""
        if self._custom_epsilon():
            return self._calc_epsilon(self.Sigma, self.K, self.T, self.dim_u)
        sigma = self.Sigma
        if sigma.shape[0] != sigma.shape[1] or sigma.shape[0] != self.dim_u or self.dim_u < 1:
            return self._calc_epsilon(sigma, self.K, self.T, self.dim_u)   # raises as the reference
        self._zbuf, self._zbuf_ev = _pinned_zbuf(getattr(self, "_zbuf", None), getattr(self, "_zbuf_ev", None),
                                                 self.K * self.T * self.dim_u)
        std = hostrng.multivariate_normal_std(np.zeros(self.dim_u), sigma, (self.K, self.T), self._zbuf.numpy())
        return std if std is not None else self._calc_epsilon(sigma, self.K, self.T, self.dim_u)

    def _drop_predraw(self):
        """Wait for a queued draw this call does not use (its buffer may be rewritten or freed next); None."""
        if self._npre is not None:
            self._settle_predraw()
        return None

    def _settle_predraw(self):
        """As MPPIControllerForPathTracking._settle_predraw."""
        pre, self._npre = self._npre, None
        new = self._npdev.result()
        return None if new is None else (pre[0], pre[1], pre[2], new)

    def _queue_predraw(self, eng: ChainEngine) -> None:
        """As MPPIControllerForPathTracking._queue_predraw: the next call's draw from the state this call's draw
        left, into this engine's second noise buffer on a stream of its own, beside this call's step (its stream
        first waits for the work already queued on the engine's, the last reader of that buffer).  The next call
        uses it when np.random is still in that state and it runs on the same engine (precision="auto" may
        switch engines: then it draws again)."""
        spec, plan = self._np_spec
        state = self._np_left
        eng._sync_stream()
        if self._noise_alt is None:
            self._noise_alt = eng.new_noise()
        if self._np_stream is None:
            self._np_stream = torch.cuda.Stream(device=eng.device)
            self._np_ev = torch.cuda.Event()
        self._np_ev.record(eng.stream)
        self._np_stream.wait_event(self._np_ev)
        rec = self._np_recorded.get(id(self._noise_alt))
        if rec is None or rec() is not self._noise_alt:   # once per tensor, as the 2-link controller
            self._noise_alt.record_stream(self._np_stream)    # its block is not reused before the draws have run
            if len(self._np_recorded) >= 4:
                self._np_recorded.clear()
            self._np_recorded[id(self._noise_alt)] = weakref.ref(self._noise_alt)
        kl = eng.K_local
        self._npdev.draw(state, (int(self.K), int(self.T), self.dim_u), plan, self._noise_alt,
                         self._np_stream.cuda_stream, eng.k_offset, kl, (self.dim_u * kl, self.dim_u, 1))
        self._npre = (state, spec, self._noise_alt)

    def _device_reference_noise(self, prec: str):
        """control.py:84 on the device, as MPPIControllerForPathTracking._device_reference_noise: NumPy's stream
        (values and RNG state) drawn into the noise buffer of the `prec` engine, the one the step runs on first
        (a step re-run in the other precision copies it over), or taken from the draw the last call queued when
        it started from NumPy's current state on this engine.  None: the host path draws."""
        from .controller import DeviceDrawn, MPPIControllerForPathTracking as _C
        if not self.numpy_noise_on_device or self._npdev is False:
            return self._drop_predraw()
        if self._custom_epsilon():
            return self._drop_predraw()
        sig = self.Sigma
        if not (isinstance(sig, np.ndarray) and sig.shape == (self.dim_u, self.dim_u)):
            return self._drop_predraw()
        n = int(self.K) * int(self.T) * self.dim_u
        if n < hostrng._MIN_NORMALS or n >= 2 ** 31:
            return self._drop_predraw()
        state = np.random.get_state()
        if state[0] != "MT19937":
            return self._drop_predraw()
        sb = sig.tobytes()
        if self._np_plan is None or self._np_plan[0] != sb or self._np_plan[1] != sig.dtype:
            self._np_plan = (sb, sig.dtype, hostrng.device_plan(np.zeros(self.dim_u), sig))
        plan = self._np_plan[2]
        if plan is None:
            return self._drop_predraw()
        self._activate(prec)
        key = self._engine_key()
        if key != self._engine_built_for:
            self._drop_predraw()                           # the engine and its buffers may be rebuilt below
            try:
                np.linalg.inv(sig)
            except np.linalg.LinAlgError:
                return None
        eng = self._get_engine(key)
        if self._npdev is None:
            try:
                from .engine import NpDeviceStream
                self._npdev = NpDeviceStream(eng.device)
            except (RuntimeError, OSError):
                self._npdev = False
                return None
        if not plan[3]:
            import warnings
            warnings.warn("covariance is not symmetric positive-semidefinite.", RuntimeWarning)   # NumPy's
        kl = eng.K_local
        spec = (int(self.K), int(self.T), self.dim_u, eng, eng.k_offset, kl, sb)
        self._np_spec = (spec, plan)
        new = None
        if self._npre is not None:
            pre = self._settle_predraw()
            if (pre is not None and pre[1] == spec and pre[2] is self._noise_alt
                    and _C._same_np_state(pre[0], state)):
                new = pre[3]                               # drawn beside the last step: NumPy's values
                self._noise_dev, self._noise_alt = self._noise_alt, self._noise_dev
                self._npre_used += 1
        if new is None:
            eng._sync_stream()
            self._npdev.draw(state, (int(self.K), int(self.T), self.dim_u), plan, self._noise_dev,
                             eng.stream.cuda_stream, eng.k_offset, kl, (self.dim_u * kl, self.dim_u, 1))  # [T][K_local][n]
            new = self._npdev.result()
        if new is None:
            return None
        np.random.set_state(new)
        self._np_left = new
        d = DeviceDrawn()
        d.buf = self._noise_dev
        return d

    def _calc_epsilon(self, sigma, size_sample, size_time_step, size_dim_u):
        """control.py:154-164 — NumPy's legacy global RNG, n-dimensional"""
        if sigma.shape[0] != sigma.shape[1] or sigma.shape[0] != size_dim_u or size_dim_u < 1:
            print("[ERROR] sigma must be a square matrix with the size of size_dim_u.")
            raise ValueError
        return hostrng.multivariate_normal(np.zeros(size_dim_u), sigma, (size_sample, size_time_step))

    def calc_control_input(self, observed_x):
        if self._npre is not None and self.noise_source != "numpy":
            self._settle_predraw()                         # (the NumPy path settles it after its checks)
        u = self.u_prev
        x0 = np.asarray(observed_x, dtype=np.float64)
        self._get_nearest_waypoint(*self._effector(x0[:self.dim_u]), update_prev_idx=True)
        if self.prev_waypoints_idx >= self.ref_path.shape[0] - 1:
            print("[ERROR] Reached the end of the reference path.")
            raise IndexError
        auto = self.precision == "auto"
        prec = ("f64" if self._spread else "f32") if auto else self.precision
        if self.noise_source == "numpy":
            epsilon = self._device_reference_noise(prec)
            if epsilon is None:
                epsilon = self._reference_noise()
            elif self.T >= 5 and not self.visualze_sampled_trajs and self.process_group is None:
                self._queue_predraw(self._engine)          # the next call's draw, beside this step
        else:
            epsilon = None
        step = self._step_count
        self._step_count += 1
        window = self.ref_path[self.prev_waypoints_idx:(self.prev_waypoints_idx + SEARCH_IDX_LEN)]
        out = self._device_step_x(prec, x0, window, u, epsilon, step)
        if auto:
            self._spread = self.last_eta - 1.0 > self.ETA_TOL
            if self._spread and prec == "f32":
                # the weights spread: this step again in fp64 from the same inputs (u is not updated yet)
                out = self._device_step_x("f64", x0, window, u, epsilon, step)
                self._spread = self.last_eta - 1.0 > self.ETA_TOL
        u_new, optimal_traj, sampled = out
        u[:] = u_new                                        # the shifted nominal, in place (aliasing kept)
        return u[0], u, optimal_traj, sampled

    def _device_step_x(self, prec: str, x0, window, u, epsilon, step: int):
        """_device_step; after an ExchangeError (raised on every rank of the step, no update applied) the same
        step again over the all-gather, which waits for the late rank, and the all-gather from then on."""
        try:
            return self._device_step(prec, x0, window, u, epsilon, step)
        except N.ExchangeError:
            # every rank re-runs the same step (a rank whose verdict differed would pair its retry with the
            # others' next step)
            if not same_on_all_ranks(("exchange retry", step), self.process_group):
                raise RuntimeError("multi-GPU exchange: the ranks disagree on the failed step; "
                                   "their nominals can no longer be kept in step") from None
            # a late rank is the ranks' property, not one engine's: every engine takes the all-gather from now on
            self._x_failed = True
            self._xmode = "rccl"
            for parked in self._slots.values():
                if parked.get("_xmode") is not None:
                    parked["_xmode"] = "rccl"
            self._noise_ready = None   # the fused step queues the next draw into the buffer: draw this one again
            return self._device_step(prec, x0, window, u, epsilon, step)

    def _device_step(self, prec: str, x0, window, u, epsilon, step: int):
        """control.py:81-149 of one step on the engine of rollout precision `prec`: the shifted updated
        nominal (T, n), the optimal trajectory and sampled_traj_list.  u (self.u_prev) is only read."""
        self._activate(prec)
        key = self._engine_key()
        if key != self._engine_built_for:
            np.linalg.inv(self.Sigma)                      # LinAlgError as control.py:106 (Sigma checked when it changes)
        eng = self._get_engine(key)
        if getattr(epsilon, "buf", None) is not None:     # a device draw (DeviceDrawn), into one engine's buffer
            if epsilon.buf is not self._noise_dev:
                eng._sync_stream()
                self._noise_dev.copy_(epsilon.buf)         # the step re-run in the other precision
        elif isinstance(epsilon, hostrng.StdNoise):
            self._zbuf_ev = eng.upload_std_noise(epsilon, self._zbuf, self._noise_dev)
        elif epsilon is not None:
            eng.upload_noise(epsilon[eng.k_offset:eng.k_offset + eng.K_local], out=self._noise_dev)
        elif self._noise_ready != (self.seed, step):
            eng.philox_noise(self.seed, step, out=self._noise_dev)
        eng.set_step_inputs(x0, window, u)
        world, _ = self._shard()
        S_out = self._S_dev if self.keep_costs else None
        if world > 1 and self._xmode is None:
            self._multi_setup(eng, _noise_check(self, epsilon))
        self.last_precision = prec
        if self.T >= 5 and not self.visualze_sampled_trajs and (world == 1 or self._xmode == "launch"):
            # the update of control.py:120-149 inside the launch (the median of 10 is a selection and the
            # add the same fp64 add: the host path's values), one read-back, the optimal trajectory in fp64
            # on the host, the next step's device noise queued behind the launch; with a process group the
            # same launch trades the ranks' rows first (the in-launch exchange)
            eng.rollout(self._noise_dev, S_out=S_out, fused_update=True, exchange=world > 1, host_out=True)
            # the next step's draw right behind the launch and its read-back (stream order: it starts once
            # the rollout has read the buffer), so it runs under the host trajectory and the caller's work
            self._prefetch_noise(eng)
            sampled = self._fresh_sampled()                     # control.py:135, while the launch runs
            u_new, traj = eng.wait_outputs(x0 if self.visualize_optimal_traj else None)
            self.last_eta = eng.last_eta()
            if self.keep_costs:
                self.last_S = self._S_dev.cpu().numpy()
            return u_new, traj if traj is not None else np.zeros((self.T, self.dim_x)), sampled
        if world == 1:
            eng.rollout(self._noise_dev, S_out=S_out)
        elif self._xmode == "launch":
            eng.rollout(self._noise_dev, S_out=S_out, exchange=True)      # one launch: rows traded in-launch
        else:
            eng.rollout(self._noise_dev, S_out=S_out, partial_out=self._partial)
            exchange_partials(self._partial, self._gathered, self.process_group)
            eng.merge(self._gathered, world)
        w_epsilon = eng.weighted_noise()
        self.last_eta = eng.last_eta()
        if self.keep_costs:
            self.last_S = self._S_dev.cpu().numpy()
        w_epsilon = np.stack([median_filter(w_epsilon[:, d], size=10, mode="reflect")
                              for d in range(self.dim_u)], axis=1)   # control.py:319-327
        un = u + w_epsilon                                            # control.py:126 (u itself untouched here)
        optimal_traj = np.zeros((self.T, self.dim_x))
        if self.visualize_optimal_traj:
            optimal_traj = eng.optimal_traj_host(x0, un)
        if self.visualze_sampled_trajs:
            tr = eng.trajectories(base_u=None, noise=self._noise_dev)
            if world > 1:
                from .distributed import gather_trajectories
                sampled = np.zeros((self.K, self.T, self.dim_x))
                gather_trajectories(tr, self.K, sampled, self.process_group)
            else:
                sampled = self._sampled_pool(tr)   # the caller's alone, as a fresh array (SampledReadback)
        else:
            sampled = np.zeros((self.K, self.T, self.dim_x))
        self._prefetch_noise(eng)
        return np.concatenate([un[1:], un[-1:]]), optimal_traj, sampled   # control.py:148-149

    def _fresh_sampled(self) -> np.ndarray:
        """A fresh writable np.zeros for sampled_traj_list (1.9 GB at config 5, mapped lazily), made while the
        launch runs; the previous call's array is kept until then, so unmapping it, if the caller dropped it,
        also happens under the launch rather than after the call returns."""
        out = np.zeros((self.K, self.T, self.dim_x))
        self._last_sampled = out
        return out

    def _prefetch_noise(self, eng: ChainEngine) -> None:
        """Device noise: the next step's draw, queued behind every reader of this step's (the
        draw is 470 MB at config 5, ~0.1 ms: off the next call's path when the caller works between calls)."""
        if self.noise_source == "device":
            eng.philox_noise(self.seed, self._step_count, out=self._noise_dev)
            self._noise_ready = (self.seed, self._step_count)

    def _close_active(self):
        if self._engine is not None:
            self._engine.close()
            self._engine = None
        self._engine_built_for = None
        self._noise_ready = None       # a new engine's noise buffer is fresh: draw again
        self._xmode = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            if self._npre is not None:
                self._settle_predraw()                     # a queued draw still writes _noise_alt
        except Exception:
            pass

    def close(self):
        if self._npre is not None:
            self._settle_predraw()                         # its buffer outlives it
        if self._npdev:
            self._npdev.close()
        self._npdev = None
        self._close_active()
        for parked in self._slots.values():
            if parked.get("_engine") is not None:
                parked["_engine"].close()
        self._slots = {}
        self._sampled_pool.clear()
