"""Drop-in ``MPPIControllerForPathTracking`` backed by the MI355X engine.

Same constructor arguments (control.py:21-35, including the ``visualze``
spelling), same ``calc_control_input(observed_x)`` contract (control.py:67-152):

  * host, fp64 NumPy (O(T) work, exactly as the reference):
      nearest-waypoint update + end-of-path ``IndexError`` (control.py:75-78),
      noise draw ``np.random.multivariate_normal`` on the legacy global RNG
      (control.py:154-164, same stream as the reference; its standard-normal
      stream threaded in C with the same values, ``hostrng``),
      ``np.linalg.inv(Sigma)`` (``LinAlgError`` as at control.py:106),
      and the aliasing return (``u0`` is a view of the shifted ``u_prev``;
      ``u_seq is self.u_prev``);
  * device, HIP (O(K*T) work): rollouts, costs, soft-min weights, weighted
    noise sum (control.py:81-118) and the trajectory re-rolls
    (control.py:129-145);
  * the update of control.py:120-149 (median filter, ``u += w_eps``, shift):
    for T >= 5 inside the rollout launch (fused update: the median of 10 is a
    selection and the add is the same fp64 add, so the values equal the host
    path's), then one read-back of the shifted nominal and the optimal
    trajectory; with T < 5, or ``host_update=True``, on the host through
    ``scipy.ndimage.median_filter`` (control.py:319-327) as the reference does.
    With device noise the next step's noise is generated at the end of a call,
    off the next call's critical path.

Extra keyword arguments (all optional): ``device``, ``verbose`` (the three
progress prints of control.py:227-229, on by default like the reference),
``noise`` ("numpy" = reference RNG stream, or "device" = on-device Philox),
``seed`` (device noise), ``lanes_per_sample``, ``arm`` (ArmParams; its
``fk_l1``/``fk_l2`` start ``self.l1``/``self.l2``, which the engine follows
from then on), ``process_group`` (shard the samples over the ranks of a
torch.distributed group), ``exchange`` (with a process group: "auto" = the
in-launch exchange, one launch per rank per step, when its one-step self-check
against the all-gather passes, else one RCCL all-gather of the per-device
partials plus a merge launch per step; "launch" or "rccl" force one) and
``host_update`` (force the host update path).

Multi-GPU: every rank constructs the controller with the same arguments and
calls ``calc_control_input`` with the same ``observed_x`` in the same order
(run.py's loop, replicated); with NumPy noise every rank draws the reference's
full (K, T, 2) stream from the same seed and keeps its slice (checked once,
at the first step).
"""
from __future__ import annotations

import sys
import weakref
from typing import Tuple

import numpy as np
import torch
from scipy.ndimage import median_filter

import dataclasses

from . import _native, hostrng
from .distributed import attach_exchange, check_exchange, exchange_partials, same_on_all_ranks, shard_geometry
from .engine import RolloutEngine
from .params import ArmParams

SEARCH_IDX_LEN = 30  # control.py:203


def first_min_index(d: np.ndarray) -> int:
    """``d.index(min(d))`` of control.py:213-215 on a 1-D array: Python's min()
    keeps d[0] and replaces it only on a strict '<', so a NaN at j > 0 is never
    chosen and a NaN at j = 0 is (np.argmin would return the first NaN)."""
    j = int(np.argmin(d))
    if d[j] != d[j]:                                   # a NaN somewhere: Python's rule
        j = 0 if d[0] != d[0] else int(np.nanargmin(d))
    return j


def _pinned_zbuf(buf, ev, n: int):
    """(buffer, None): a float64 host tensor of at least n values, page-locked where the host allows it,
    reused across calls once the event of the last DMA out of it has completed."""
    if ev is not None:
        ev.synchronize()
    if buf is None or buf.numel() < n:
        buf = None   # the old one is released first
        try:
            buf = torch.empty(n, dtype=torch.float64, pin_memory=True)
        except RuntimeError:
            buf = torch.empty(n, dtype=torch.float64)
    return buf, None


class DeviceDrawn:
    """The reference's draw (control.py:84) made on the device straight into the engine's noise buffer
    (engine.NpDeviceStream)."""


def _noise_check(ctrl, epsilon):
    """The value the ranks compare at their first step to agree on the noise stream.  The reference's own draw
    (NumPy's global RNG, control.py:163): the RNG state it left, which the device draw and the host draw leave
    alike, so a rank that fell back to the host draw still agrees with one that drew on the device; a replaced
    _calc_epsilon: eps[0, 0, 0] + eps[-1, -1, -1] of its array; device noise: None (the seed is compared)."""
    if ctrl.noise_source != "numpy" or epsilon is None:
        return None
    if not ctrl._custom_epsilon():
        st = np.random.get_state()
        return (float(np.sum(np.asarray(st[1][:16], dtype=np.float64))), int(st[2]), int(st[3]), float(st[4]))
    if isinstance(epsilon, hostrng.StdNoise):
        K, T, du = epsilon.z.shape
        return epsilon.eps(0, 0, 0) + epsilon.eps(K - 1, T - 1, du - 1)
    return float(epsilon[0, 0, 0] + epsilon[-1, -1, -1])


class SampledReadback:
    """sampled_traj_list's host arrays (control.py:135-145): the device re-roll's fp32 states read back and
    widened to fp64 on the host (engine.HostReadback: chunked DMA of the fp32 bytes, host threads widening
    each landed chunk; fp32 -> fp64 is exact, so the values are the device-side widening's, with half the
    bytes over the host link: 2.5 -> ~1.3 ms at K = 65536, T = 64) into an array of a pool that no caller
    holds any more, returned as is.  An array is reused only when nothing outside the pool refers to it (views
    of it included: their base is that array), so every returned array is the caller's alone, as
    control.py:137's fresh np.zeros is; a reused array's pages are already mapped.

    The pool is bounded: at most MAX arrays and MAX_BYTES in all (a larger array, e.g. the chain's 1.9 GB at
    config 5, is a fresh one per call).  A CPU tensor (tests) is widened by torch."""

    MAX = 3                 # arrays held at most (run.py's loop holds one array across a call: it cycles through two)
    MAX_BYTES = 768 << 20   # bytes held at most (3 x 134 MB at K = 65536, T = 64 fit)

    def __init__(self):
        self._pool = []    # arrays
        self._rb = None    # engine.HostReadback of the device last read from

    def clear(self) -> None:
        self._pool = []    # arrays the caller still holds stay theirs
        if self._rb is not None:
            self._rb.close()
            self._rb = None

    def __len__(self) -> int:
        return len(self._pool)

    def _fill(self, tr: torch.Tensor, out: np.ndarray) -> np.ndarray:
        if not tr.is_cuda:
            np.copyto(out, tr.double().numpy())
            return out
        if self._rb is None or self._rb.device != tr.device:
            from .engine import HostReadback
            if self._rb is not None:
                self._rb.close()
            self._rb = HostReadback(tr.device)
        return self._rb.run(tr.contiguous(), out)

    def __call__(self, tr: torch.Tensor) -> np.ndarray:
        shape = tuple(tr.shape)
        pool = self._pool
        if pool and tuple(pool[0].shape) != shape:
            self._pool = pool = []   # K or T changed
        for arr in pool:
            if sys.getrefcount(arr) == 3:   # the pool list's reference, the loop variable's and the argument's
                return self._fill(tr, arr)
        arr = np.empty(shape)
        if len(pool) < self.MAX and (len(pool) + 1) * arr.nbytes <= self.MAX_BYTES:
            pool.append(arr)
        return self._fill(tr, arr)


class MPPIControllerForPathTracking:
    def __init__(
            self,
            delta_t: float = 0.01,
            ref_path: float = 0,
            horizon_step_T: int = 20,
            number_of_samples_K: int = 500,
            param_exploration: float = 0.0,
            param_lambda: float = 50.0,
            param_alpha: float = 1.0,
            sigma: np.ndarray = np.array([[10.0, 10.0], [100.0, 100.0]]),
            stage_cost_weight: np.ndarray = np.array([10.0, 10.0, 10.0, 10.0]),
            terminal_cost_weight: np.ndarray = np.array([10.0, 10.0, 10.0, 10.0]),
            visualize_optimal_traj=True,
            visualze_sampled_trajs=False,
            *,
            device: int | None = None,
            verbose: bool = True,
            noise: str = "numpy",
            seed: int = 0,
            lanes_per_sample: int = 0,
            arm: ArmParams | None = None,
            process_group=None,
            exchange: str = "auto",
            host_update: bool = False,
            numpy_noise_on_device: bool = True,
    ) -> None:
        self.dim_x = 4
        self.dim_u = 2
        self.T = horizon_step_T
        self.K = number_of_samples_K
        self.param_exploration = param_exploration
        self.param_lambda = param_lambda
        self.param_alpha = param_alpha
        self.param_gamma = self.param_lambda * (1.0 - (self.param_alpha))
        self.Sigma = sigma
        self.stage_cost_weight = stage_cost_weight
        self.terminal_cost_weight = terminal_cost_weight
        self.visualize_optimal_traj = visualize_optimal_traj
        self.visualze_sampled_trajs = visualze_sampled_trajs
        self.delta_t = delta_t
        self.ref_path = ref_path
        self.l1 = 1
        self.l2 = 1
        self.u_prev = np.array([[10.0, -2.0] for i in range(self.T)])
        self.prev_waypoints_idx = 0

        if noise not in ("numpy", "device"):
            raise ValueError("noise must be 'numpy' or 'device'")
        self.verbose = verbose
        self.noise_source = noise
        self.seed = int(seed)
        if arm is not None:                # the cost's kinematics lengths (control.py:55-56)
            self.l1, self.l2 = arm.fk_l1, arm.fk_l2
        self.arm = ArmParams(fk_l1=float(self.l1), fk_l2=float(self.l2)) if arm is None else arm
        self.process_group = process_group
        if exchange not in ("auto", "launch", "rccl"):
            raise ValueError("exchange must be 'auto', 'launch' or 'rccl'")
        self.exchange = exchange
        self._xmode = None             # multi-GPU exchange in use: "launch" / "rccl" (decided at the first step)
        self._x_failed = False         # an in-launch exchange failed (a late rank): the all-gather for good
        self._lanes_per_sample = lanes_per_sample
        self._device = device
        self._engine = None
        self._step_count = 0
        self._noise_ready = None       # (seed, step) of the device noise already in the buffer
        self._engine_built_for = None  # _engine_key() of the live engine
        self.host_update = host_update  # property: forced, or T < 5 (the device median needs T >= 5)
        self.keep_costs = False        # set True to keep per-sample S (self.last_S)
        self.last_S = None
        self._bound = None             # what the engine's drop-in tick is bound to (_bind_key)
        self._last_sampled = None      # the previous call's sampled_traj_list (_fresh_sampled)
        self._sampled_pool = SampledReadback()   # sampled_traj_list's read-back arrays (_sampled_host)
        self._fast = None              # what the last bound tick checked (calc_control_input's fast test)
        self.numpy_noise_on_device = numpy_noise_on_device   # noise="numpy": the same stream drawn on the device
        self._npdev = None             # its engine.NpDeviceStream (False: unavailable here)
        self._npre = None              # (start state, spec) of the next call's draw, queued at the end of a call
        self._np_spec = None           # (spec, plan) of this call's device draw
        self._npre_used = 0            # calls that used the queued draw
        self._np_queued = False        # this call queued the next call's draw already
        self._np_recorded = {}         # id -> weakref of the noise buffers already record_stream'ed on the draw stream
        self._np_plan = None           # (Sigma bytes, dtype, hostrng.device_plan) of the last draw
        self._np_left = None           # the state this call's draw left np.random in
        self._noise_alt = None         # the second noise buffer: the queued draw writes it while a step reads the other
        self._np_stream = None         # the stream of the queued draws (concurrent with the step)
        self._np_ev = None

    @property
    def host_update(self) -> bool:
        """The update of control.py:120-149 on the host: asked for, or T < 5 (the
        device median filter needs T >= 5), following self.T if it changes."""
        return self._host_update or self.T < 5

    @host_update.setter
    def host_update(self, value) -> None:
        self._host_update = bool(value)

    # ------------------------------------------------------------ engine
    def _shard(self):
        if self.process_group is None:
            return 1, 0
        import torch.distributed as dist
        return dist.get_world_size(self.process_group), dist.get_rank(self.process_group)

    def _engine_key(self):
        """Everything the engine bakes in at creation that the reference reads on
        every call (Sigma at control.py:84,106; lambda :112; gamma :106; the cost
        weights :185,198; the exploration split :98; delta_t :256-259; the
        kinematics lengths self.l1/l2 of :178-179,205-206; the arm constants; the
        sample count and horizon self.K / self.T of :81-95)."""
        return (int(self.K), int(self.T), np.asarray(self.Sigma, dtype=np.float64).tobytes(), float(self.param_lambda),
                float(self.param_gamma), np.asarray(self.stage_cost_weight, dtype=np.float64).tobytes(),
                np.asarray(self.terminal_cost_weight, dtype=np.float64).tobytes(), float(self.param_exploration),
                float(self.delta_t), float(self.l1), float(self.l2), self.arm)

    def _get_engine(self, key=None) -> RolloutEngine:
        key = self._engine_key() if key is None else key
        if self._engine is not None and key != self._engine_built_for:
            self.close()             # an attribute the engine baked in changed: rebuild, as the reference re-reads it
        if self._engine is None:
            world, rank = self._shard()
            K_local, k_offset = shard_geometry(self.K, world, rank)
            device = self._device if self._device is not None else torch.cuda.current_device()
            # gamma is fixed at construction in the reference (control.py:45) while lambda is
            # re-read per call: the engine takes gamma as given; the cost's kinematics follow self.l1/l2
            arm = dataclasses.replace(self.arm, fk_l1=float(self.l1), fk_l2=float(self.l2))
            self._engine = RolloutEngine(
                K_local, self.T, self.delta_t, self.param_lambda, self.param_alpha, self.Sigma,
                self.stage_cost_weight, self.terminal_cost_weight, self.param_exploration, arm,
                K_total=self.K, k_offset=k_offset, device=device, lanes_per_sample=self._lanes_per_sample,
                param_gamma=self.param_gamma)
            self._engine_built_for = key
            self._noise_dev = self._engine.new_noise()
            self._noise_alt = None
            self._partial = self._engine.new_partial()
            self._S_dev = torch.empty(K_local, dtype=torch.float64, device=self._engine.device)
            self._traj_dev = torch.empty((self.T, self.dim_x), dtype=torch.float32, device=self._engine.device)
            if world > 1:
                self._gathered = torch.empty(world * self._engine.partial_len, dtype=torch.float64,
                                             device=self._engine.device)
            self._xmode = None
        return self._engine

    def _multi_setup(self, eng: RolloutEngine, noise_check) -> None:
        """First multi-GPU step of an engine (collective, every rank): check that the
        ranks agree on the noise stream, then pick the exchange — the in-launch one
        (distributed.attach_exchange) if its one-step self-check against the
        all-gather + merge passes (distributed.check_exchange), else RCCL."""
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

    def _multi_rollout(self, eng: RolloutEngine, S_out, fused: bool) -> None:
        """control.py:81-118 over every rank's shard, the rows merged on every rank:
        one launch with the in-launch exchange, or rollout + RCCL all-gather + merge
        launch.  fused: the update of control.py:120-149 too, published for wait_outputs."""
        if self._xmode == "launch":
            eng.rollout(self._noise_dev, S_out=S_out, fused_update=fused, exchange=True, host_out=fused)
            return
        world, _ = self._shard()
        eng.rollout(self._noise_dev, S_out=S_out, partial_out=self._partial)
        exchange_partials(self._partial, self._gathered, self.process_group)
        eng.merge(self._gathered, world, fused_update=fused, host_out=fused)

    # ------------------------------------------------------------ API
    def calc_control_input(self, observed_x: np.ndarray) -> Tuple[float, np.ndarray]:
        """calculate optimal control input (control.py:67-152)"""
        if self.process_group is not None and (self._xmode == "launch" or (
                self._xmode is None and self.exchange != "rccl" and not self._x_failed)):
            # the in-launch exchange can fail on a late rank (ExchangeError on every rank of the step, no update
            # applied anywhere): every rank then restores what the call changed and runs it again over the
            # all-gather, which waits for the late rank, and stays on it.  The first call is covered too (it
            # picks the exchange and then runs its step in-launch).
            saved = (self.prev_waypoints_idx, self._step_count,
                     np.random.get_state() if self.noise_source == "numpy" else None)
            try:
                return self._calc_control_input(observed_x)
            except _native.ExchangeError:
                self.prev_waypoints_idx, self._step_count, rng = saved
                # the ranks re-run the same step: a rank whose verdict differed (it saw the step fail while the
                # others applied it) would pair its retry's all-gather with their next step
                if not same_on_all_ranks(("exchange retry", self._step_count), self.process_group):
                    raise RuntimeError("multi-GPU exchange: the ranks disagree on the failed step; "
                                       "their nominals can no longer be kept in step") from None
                if rng is not None:
                    np.random.set_state(rng)
                self._exchange_failed()
                verbose, self.verbose = self.verbose, False     # the call's three lines are printed already
                try:
                    return self._calc_control_input(observed_x)
                finally:
                    self.verbose = verbose
        return self._calc_control_input(observed_x)

    def _exchange_failed(self) -> None:
        """After an ExchangeError (every rank): the collective exchange from now on, no native tick, and the
        device noise drawn again for the step (the tick queues the next step's draw into the same buffer)."""
        self._xmode = "rccl"
        self._x_failed = True
        self._fast = None
        self._bound = None
        self._noise_ready = None

    def _calc_control_input(self, observed_x: np.ndarray) -> Tuple[float, np.ndarray]:
        if self._npre is not None and self.noise_source != "numpy":
            self._settle_predraw()                         # (the NumPy path settles it after its checks)
        f = self._fast
        if (f is not None and f[0] is self.ref_path and f[1] is self.u_prev and f[2] is self.Sigma
                and f[3] is self.stage_cost_weight and f[4] is self.terminal_cost_weight and f[5] is self._engine
                and f[6] == self._fast_scalars() and f[7] == self.Sigma.tobytes()
                and f[8] == self.stage_cost_weight.tobytes() and f[9] == self.terminal_cost_weight.tobytes()):
            return self._tick_bound(observed_x)
        if (self.noise_source == "device" and not self.host_update and not self.visualze_sampled_trajs
                and (self.process_group is None or self._xmode == "launch") and self.K >= 1):
            out = self._tick(observed_x)
            if out is not None:
                return out
        u = self.u_prev
        x0 = observed_x
        self._get_nearest_waypoint(x0[0], x0[1], update_prev_idx=True)
        if self.prev_waypoints_idx >= self.ref_path.shape[0] - 1:
            print("[ERROR] Reached the end of the reference path.")
            raise IndexError
        if self.K < 1:
            raise ValueError("zero-size array to reduction operation minimum which has no identity")

        if self.noise_source == "numpy":
            epsilon = self._device_reference_noise()
            if epsilon is None:
                epsilon = self._reference_noise()
        else:
            epsilon = None
            self._check_sigma(self.Sigma, self.dim_u)
        key = self._engine_key()
        if key != self._engine_built_for:
            np.linalg.inv(self.Sigma)                      # LinAlgError exactly as control.py:106
        eng = self._get_engine(key)
        if isinstance(epsilon, DeviceDrawn):
            pass                                           # already in self._noise_dev
        elif isinstance(epsilon, hostrng.StdNoise):
            self._zbuf_ev = eng.upload_std_noise(epsilon, self._zbuf, self._noise_dev)
        elif epsilon is not None:
            lo = eng.k_offset
            eng.upload_noise(epsilon[lo:lo + eng.K_local], out=self._noise_dev)
        elif self._noise_ready != (self.seed, self._step_count):
            eng.philox_noise(self.seed, self._step_count, out=self._noise_dev)
        self._step_count += 1

        window = self.ref_path[self.prev_waypoints_idx:(self.prev_waypoints_idx + SEARCH_IDX_LEN)]
        world, _ = self._shard()
        if not self.host_update and world == 1 and not self.visualze_sampled_trajs:
            if isinstance(epsilon, DeviceDrawn) and not self._np_queued:
                self._queue_predraw(eng)                   # the next call's draw, beside this step
            self._np_queued = False
            return self._dropin_step(eng, x0, window, u)
        eng.set_step_inputs(np.asarray(x0, dtype=np.float64), window, u)
        if world > 1 and self._xmode is None:
            check = _noise_check(self, epsilon)
            self._multi_setup(eng, check)
        if not self.host_update:
            return self._fused_step(eng, x0, u, world, predraw=isinstance(epsilon, DeviceDrawn) and world == 1)
        S_out = self._S_dev if self.keep_costs else None
        if world == 1:
            eng.rollout(self._noise_dev, S_out=S_out)
        else:
            self._multi_rollout(eng, S_out, fused=False)
        w_epsilon = eng.weighted_noise()
        if self.keep_costs:
            self.last_S = self._S_dev.cpu().numpy()

        w_epsilon = self._moving_median_filter(xx=w_epsilon, window_size=10)
        u += w_epsilon

        optimal_traj = np.zeros((self.T, self.dim_x))
        if self.visualize_optimal_traj:
            optimal_traj = eng.optimal_traj_host(x0, u)

        if self.visualze_sampled_trajs:
            tr = eng.trajectories(base_u=None, noise=self._noise_dev)   # pre-update u, v[k, t-1]
            sampled_traj_list = self._sampled_host(tr, world)
        else:
            sampled_traj_list = np.zeros((self.K, self.T, self.dim_x))

        self.u_prev[:-1] = u[1:]
        self.u_prev[-1] = u[-1]
        self._prefetch_noise(eng)
        return u[0], u, optimal_traj, sampled_traj_list

    def _sampled_host(self, tr: torch.Tensor, world: int) -> np.ndarray:
        """sampled_traj_list (K, T, 4) fp64 (control.py:135-145) from the device re-roll: widened to fp64 on
        the device and read back into a host array that is returned as is (no second 134 MB copy into an
        np.zeros; SampledReadback); the ranks' shards gathered into one array with a process group."""
        if world > 1:
            from .distributed import gather_trajectories
            out = np.zeros((self.K, self.T, self.dim_x))
            gather_trajectories(tr, self.K, out, self.process_group)
            return out
        return self._sampled_pool(tr)

    def _fresh_sampled(self) -> np.ndarray:
        """A fresh writable zero array for sampled_traj_list (control.py:137: np.zeros each call, 134 MB at
        K = 65536, T = 64), made while the launch runs.  The controller keeps the previous call's array until
        now, so if the caller has dropped it, its unmapping (~12 us) also happens here, under the launch,
        instead of in the caller after the call returns; an array the caller still holds is untouched."""
        out = np.zeros((self.K, self.T, self.dim_x))
        self._last_sampled = out
        return out

    def _tick(self, observed_x):
        """The whole call in one native step (mppi_dropin_tick) when the buffers it
        binds are plain arrays: the fp64 nearest-waypoint update and end-of-path
        check of control.py:70-78 (the same operations as _get_nearest_waypoint),
        then the fused device step of _dropin_step.  None: not applicable, take the
        general path."""
        path, u = self.ref_path, self.u_prev
        if not (isinstance(path, np.ndarray) and path.dtype == np.float64 and path.ndim == 2 and path.shape[1] >= 4
                and path.strides[1] == 8 and path.strides[0] % 8 == 0 and path.strides[0] >= 32
                and isinstance(u, np.ndarray) and u.dtype == np.float64
                and u.shape == (self.T, 2) and u.flags.c_contiguous and u.flags.writeable):
            return None
        sig = self.Sigma
        if not (isinstance(sig, np.ndarray) and sig.shape == (self.dim_u, self.dim_u)):
            return None                                    # the general path raises as the reference does
        key = self._engine_key()
        if self._engine is None or key != self._engine_built_for:
            return None                                    # (re)build on the general path (LinAlgError order kept)
        eng = self._engine
        bkey = (eng, path, u, self.keep_costs, self.visualize_optimal_traj, self.seed, self.l1, self.l2,
                self._noise_dev)                           # (a NumPy-noise run swaps the noise buffers)
        if self._bound is None or any(a is not b for a, b in zip(bkey, self._bound)):
            self._x_buf = np.zeros(4)
            self._idx_buf = np.zeros(2, dtype=np.int64)
            self._traj_buf = np.zeros((self.T, self.dim_x)) if self.visualize_optimal_traj else None
            eng.dropin_bind(path, float(self.l1), float(self.l2), self._x_buf, self._idx_buf, u, self._traj_buf,
                            self._noise_dev, self._noise_dev, self._S_dev if self.keep_costs else None, self.seed)
            self._bound = bkey
        if self._noise_ready != (self.seed, self._step_count):
            eng.philox_noise(self.seed, self._step_count, out=self._noise_dev)
        out = self._tick_bound(observed_x)
        # the next call may skip every check above while nothing they read has changed
        # (the same objects, scalars and array contents): calc_control_input's fast test
        if all(isinstance(a, np.ndarray) and a.dtype == np.float64
               for a in (self.Sigma, self.stage_cost_weight, self.terminal_cost_weight)):
            self._fast = (path, u, self.Sigma, self.stage_cost_weight, self.terminal_cost_weight, eng,
                          self._fast_scalars(), self.Sigma.tobytes(), self.stage_cost_weight.tobytes(),
                          self.terminal_cost_weight.tobytes())
        return out

    def _fast_scalars(self):
        """Every scalar _tick's checks and the engine key read (control.py's per-call reads of
        lambda, gamma, the exploration split, delta_t, l1/l2), plus the controller switches."""
        return (self.noise_source, self.host_update, self.visualze_sampled_trajs, self.process_group, self.K, self.T,
                self.param_lambda, self.param_gamma, self.param_exploration, self.delta_t, self.l1, self.l2,
                self.arm, self.seed, self.keep_costs, self.visualize_optimal_traj, self.verbose,
                self._noise_ready == (self.seed, self._step_count))

    def _tick_bound(self, observed_x):
        """The bound drop-in tick (engine built, buffers bound, the noise of this step in
        the buffer): stage x0 and the index, launch, allocate sampled_traj_list, wait."""
        eng = self._engine
        if type(observed_x) is np.ndarray and observed_x.shape == (4,):
            self._x_buf[:] = observed_x
        else:
            self._x_buf[:] = np.asarray(observed_x, dtype=np.float64).ravel()[:4]
        self._idx_buf[0] = self.prev_waypoints_idx
        self._step_count += 1
        rc = eng.dropin_tick_launch(self._step_count)
        self.prev_waypoints_idx = self._idx_buf.item(0)
        if rc != 0:                                        # MPPI_E_PATH_END: nothing was launched
            if self.verbose:
                self._print_update(int(self._idx_buf[1]), self.prev_waypoints_idx)
            self._step_count -= 1
            print("[ERROR] Reached the end of the reference path.")
            raise IndexError
        # the launched step is always consumed (its wait runs whatever is raised in between: a failing
        # print or allocation, KeyboardInterrupt), so the next launch never finds a tick still pending
        try:
            if self.verbose:
                self._print_update(int(self._idx_buf[1]), self.prev_waypoints_idx)
            sampled = self._fresh_sampled()                 # control.py:135, allocated while the launch runs
        finally:
            eng.dropin_tick_wait()
        self._noise_ready = (self.seed, self._step_count)
        if self.keep_costs:
            self.last_S = self._S_dev.cpu().numpy()
        traj = self._traj_buf.copy() if self._traj_buf is not None else np.zeros((self.T, self.dim_x))
        u = self.u_prev
        return u[0], u, traj, sampled

    def _dropin_step(self, eng: RolloutEngine, x0, window, u: np.ndarray):
        """control.py:81-152 on one device in one native call (mppi_step_dropin):
        rollouts + soft-min + weighted noise + median filter + u += w_eps + shift in
        the launch, the result read from host-mapped memory, the optimal trajectory
        in fp64 on the host from the update, then the next step's device noise queued
        behind the rollout.  u is self.u_prev (updated in place)."""
        nxt = self._noise_dev if self.noise_source == "device" else None
        u_new, traj = eng.step_dropin(x0, window, u, self._noise_dev,
                                      S_out=self._S_dev if self.keep_costs else None, next_noise=nxt,
                                      seed=self.seed, next_step=self._step_count,
                                      want_traj=self.visualize_optimal_traj)
        if nxt is not None:
            self._noise_ready = (self.seed, self._step_count)
        if self.keep_costs:
            self.last_S = self._S_dev.cpu().numpy()
        u[:] = u_new                                       # the shifted nominal, in place (aliasing kept)
        optimal_traj = traj if traj is not None else np.zeros((self.T, self.dim_x))
        return u[0], u, optimal_traj, self._fresh_sampled()

    def _fused_step(self, eng: RolloutEngine, x0, u: np.ndarray, world: int, predraw: bool = False):
        """control.py:81-152 with the update inside the launch (the multi-GPU merge
        launch, or the rollout when sampled trajectories are asked for): median filter
        + u += w_eps + shift on device, the result read from host-mapped memory, the
        optimal trajectory in fp64 on the host from the update.  u is self.u_prev
        (updated in place).  predraw: the next call's NumPy draw is queued behind the
        trajectory re-roll, so it runs during the sampled trajectories' read-back."""
        S_out = self._S_dev if self.keep_costs else None
        u_before = u.copy() if self.visualze_sampled_trajs else None
        if world == 1:
            eng.rollout(self._noise_dev, S_out=S_out, fused_update=True, host_out=True)
        else:
            self._multi_rollout(eng, S_out, fused=True)
        tr = None
        if self.visualze_sampled_trajs:
            tr = eng.trajectories(base_u=u_before, noise=self._noise_dev)   # pre-update u, v[k, t-1]
        if predraw:
            self._queue_predraw(eng)
        u_new, traj = eng.wait_outputs(x0 if self.visualize_optimal_traj else None)
        if self.keep_costs:
            self.last_S = self._S_dev.cpu().numpy()
        sampled_traj_list = (self._sampled_host(tr, world) if tr is not None
                             else np.zeros((self.K, self.T, self.dim_x)))
        # next step's noise after the last read-back: the draw overlaps the caller's
        # work between ticks instead of sitting in front of this call's wait
        self._prefetch_noise(eng)
        u[:] = u_new                                       # the shifted nominal, in place (aliasing kept)
        optimal_traj = traj if traj is not None else np.zeros((self.T, self.dim_x))
        return u[0], u, optimal_traj, sampled_traj_list

    def _prefetch_noise(self, eng: RolloutEngine) -> None:
        """Device noise: draw the next step's noise now (stream-ordered after every
        reader of this step's), so the next call does not wait for it."""
        if self.noise_source == "device":
            eng.philox_noise(self.seed, self._step_count, out=self._noise_dev)
            self._noise_ready = (self.seed, self._step_count)

    # ------------------------------------------------------------ host helpers (reference semantics)
    @staticmethod
    def _check_sigma(sigma, size_dim_u):
        if sigma.shape[0] != sigma.shape[1] or sigma.shape[0] != size_dim_u or size_dim_u < 1:
            print("[ERROR] sigma must be a square matrix with the size of size_dim_u.")
            raise ValueError

    def _custom_epsilon(self) -> bool:
        """_calc_epsilon replaced on the instance or a subclass: the caller's noise, not the reference's draw."""
        cls = MPPIControllerForPathTracking
        return "_calc_epsilon" in self.__dict__ or type(self)._calc_epsilon is not cls._calc_epsilon

    def _reference_noise(self):
        """control.py:84, the reference's draw on the legacy global RNG.  When _calc_epsilon is the reference's
        (not replaced on the instance or a subclass) and Sigma's transform is a scaled column permutation
        (run.py's 20 I), the draw stops at its standard normals: NumPy's values, written into a page-locked
        buffer that goes to the device in one DMA, where the same fp64 multiply and add make the noise
        (hostrng.multivariate_normal_std, engine.upload_std_noise) instead of NumPy's np.dot and `x += mean`
        over the 67 MB draw and a pageable copy.  Otherwise _calc_epsilon's array."""
        if self._custom_epsilon():
            return self._calc_epsilon(self.Sigma, self.K, self.T, self.dim_u)
        self._check_sigma(self.Sigma, self.dim_u)
        std = hostrng.multivariate_normal_std(np.full((self.dim_u), 0.0), self.Sigma, (self.K, self.T),
                                              self._zbuf_numpy(self.K * self.T * self.dim_u))
        return std if std is not None else self._calc_epsilon(self.Sigma, self.K, self.T, self.dim_u)

    def _drop_predraw(self):
        """Wait for a queued draw this call does not use (its buffer may be rewritten or freed next); None."""
        if self._npre is not None:
            self._settle_predraw()
        return None

    def _settle_predraw(self):
        """Wait for the draw queued by the last call: (the state it started from, its spec, its buffer, the state
        it leaves), or None.  Settled before anything may rewrite or free its buffer."""
        pre, self._npre = self._npre, None
        new = self._npdev.result()
        return None if new is None else (pre[0], pre[1], pre[2], new)

    def _queue_predraw(self, eng: RolloutEngine) -> None:
        """The next call's draw, queued before this call's step from the state this call's draw left, into the
        second noise buffer on a stream of its own: it runs beside the step and while the caller works between
        calls.  Its stream first waits for the work already queued on the engine's stream (the last step, which
        read that buffer).  The next call uses it only if NumPy's state is still that one and nothing the draw
        depends on has changed (_device_reference_noise); otherwise it draws again, so the values and state are
        NumPy's either way."""
        spec, plan = self._np_spec
        state = self._np_left                              # np.random's state now: this call set it last
        eng._sync_stream()
        if self._noise_alt is None:
            self._noise_alt = eng.new_noise()
        if self._np_stream is None:
            self._np_stream = torch.cuda.Stream(device=eng.device)
            self._np_ev = torch.cuda.Event()
        self._np_ev.record(eng.stream)
        self._np_stream.wait_event(self._np_ev)
        rec = self._np_recorded.get(id(self._noise_alt))
        if rec is None or rec() is not self._noise_alt:
            # its block is not reused before the draws on that stream have run (recorded once per tensor: the
            # allocator keeps the stream with the block until it is freed)
            self._noise_alt.record_stream(self._np_stream)
            if len(self._np_recorded) >= 4:
                self._np_recorded.clear()
            self._np_recorded[id(self._noise_alt)] = weakref.ref(self._noise_alt)
        self._npdev.draw(state, (int(self.K), int(self.T), self.dim_u), plan, self._noise_alt,
                         self._np_stream.cuda_stream, eng.k_offset, eng.K_local,
                         (eng.K_local * self.dim_u, self.dim_u, 1))
        self._npre = (state, spec, self._noise_alt)

    @staticmethod
    def _same_np_state(a, b) -> bool:
        return (a[0] == b[0] and a[2] == b[2] and a[3] == b[3] and a[4] == b[4]
                and np.array_equal(a[1], b[1]))

    def _device_reference_noise(self):
        """control.py:84 on the device: the reference's own stream (np.random.multivariate_normal on the legacy
        global RNG, NumPy's values and the state it leaves) drawn straight into the engine's noise buffer
        (engine.NpDeviceStream, include/mppi_rocm.h mppi_np_*), when _calc_epsilon is the reference's and Sigma's
        transform is a scaled column permutation (run.py's 20 I) or, for the 2-link arm, any matrix whose np.dot
        rounding hostrng.dot2_model pins.  None: not applicable here (the host path
        draws then; nothing was drawn).  A singular Sigma takes the host path too, which draws before
        np.linalg.inv raises, as control.py:84,106 do.  The draw the last call queued is waited for only after
        these checks (they run while it does), and used when it started from NumPy's current state."""
        if not self.numpy_noise_on_device or self._npdev is False:
            return self._drop_predraw()
        if self._custom_epsilon():
            return self._drop_predraw()
        sig = self.Sigma
        if not (isinstance(sig, np.ndarray) and sig.shape == (self.dim_u, self.dim_u)):
            return self._drop_predraw()                    # the host path prints and raises as the reference
        n = int(self.K) * int(self.T) * self.dim_u
        if n < hostrng._MIN_NORMALS or n >= 2 ** 31:
            return self._drop_predraw()
        state = np.random.get_state()
        if state[0] != "MT19937":
            return self._drop_predraw()
        sb = sig.tobytes()
        if self._np_plan is None or self._np_plan[0] != sb or self._np_plan[1] != sig.dtype:
            self._np_plan = (sb, sig.dtype, hostrng.device_plan(np.full((self.dim_u), 0.0), sig))
        plan = self._np_plan[2]
        if plan is None:
            return self._drop_predraw()
        key = self._engine_key()
        if key != self._engine_built_for:
            self._drop_predraw()                           # the engine and its buffer may be rebuilt below
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
        spec = (int(self.K), int(self.T), self.dim_u, eng, eng.k_offset, eng.K_local, sb)
        self._np_spec = (spec, plan)
        new = None
        if self._npre is not None:
            pre = self._settle_predraw()
            if (pre is not None and pre[1] == spec and pre[2] is self._noise_alt
                    and self._same_np_state(pre[0], state)):
                new = pre[3]                               # drawn beside the last step: NumPy's values
                self._noise_dev, self._noise_alt = self._noise_alt, self._noise_dev
                self._npre_used += 1
        if new is None:
            eng._sync_stream()
            self._npdev.draw(state, (int(self.K), int(self.T), self.dim_u), plan, self._noise_dev,
                             eng.stream.cuda_stream, eng.k_offset, eng.K_local, (eng.K_local * self.dim_u, self.dim_u, 1))
            new = self._npdev.result()
        if new is None:
            return None
        self._np_left = new
        if not self.host_update and not self.visualze_sampled_trajs and self._shard()[0] == 1:
            self._queue_predraw(eng)                       # the next call's draw, now: the device is idle until
            self._np_queued = True                         # it is queued (the step follows on its own stream)
        np.random.set_state(new)
        return DeviceDrawn()

    def _zbuf_numpy(self, n: int) -> np.ndarray:
        """The page-locked buffer of the standard normals (>= n values), free to be rewritten: the DMA of the
        previous draw out of it has completed."""
        self._zbuf, self._zbuf_ev = _pinned_zbuf(getattr(self, "_zbuf", None), getattr(self, "_zbuf_ev", None), n)
        return self._zbuf.numpy()

    def _calc_epsilon(self, sigma: np.ndarray, size_sample: int, size_time_step: int, size_dim_u: int) -> np.ndarray:
        """sample epsilon (control.py:154-164) — the reference's RNG stream"""
        self._check_sigma(sigma, size_dim_u)
        mu = np.full((size_dim_u), 0.0)
        return hostrng.multivariate_normal(mu, sigma, (size_sample, size_time_step))   # NumPy's values, threaded

    def _g(self, v: np.ndarray) -> float:
        """clamp input (disabled in the reference, control.py:166-172)"""
        return v

    def _get_nearest_waypoint(self, q1: float, q2: float, update_prev_idx: bool = False):
        """search the closest waypoint (control.py:200-232), host fp64"""
        prev_idx = self.prev_waypoints_idx
        x = self.l1 * np.cos(q1) + self.l2 * np.cos(q1 + q2)
        y = self.l1 * np.sin(q1) + self.l2 * np.sin(q1 + q2)
        win = self.ref_path[prev_idx:(prev_idx + SEARCH_IDX_LEN)]
        d = ((x - win[:, 0]) ** 2 + (y - win[:, 1]) ** 2) * 100
        nearest_idx = first_min_index(d) + prev_idx
        ref_x = self.ref_path[nearest_idx, 0]
        ref_y = self.ref_path[nearest_idx, 1]
        ref_dq1 = self.ref_path[nearest_idx, 2]
        ref_dq2 = self.ref_path[nearest_idx, 3]
        if update_prev_idx:
            if self.verbose:
                self._print_update(prev_idx, nearest_idx)
            self.prev_waypoints_idx = nearest_idx
        return nearest_idx, ref_x, ref_y, ref_dq1, ref_dq2

    @staticmethod
    def _print_update(prev_idx: int, nearest_idx: int) -> None:
        """the three progress lines of control.py:227-229"""
        print(f"0     prev_idx = {prev_idx}")
        print(f"0     nearest_idx = {nearest_idx}")
        print("======================updated=======================")

    def _moving_median_filter(self, xx: np.ndarray, window_size: int) -> np.ndarray:
        """median smoothing per input dimension (control.py:319-327)"""
        out = np.zeros(xx.shape)
        for d in range(xx.shape[1]):
            out[:, d] = median_filter(xx[:, d], size=window_size, mode='reflect')
        return out

    def __del__(self):  # pragma: no cover - best effort
        try:
            if self._npre is not None:
                self._settle_predraw()                     # a queued draw still writes _noise_alt
        except Exception:
            pass

    def close(self):
        if self._npre is not None:
            self._settle_predraw()                         # its buffer outlives it
        if self._engine is not None:
            self._engine.close()
            self._engine = None
        if self._npdev:
            self._npdev.close()
        self._npdev = None
        self._noise_ready = None       # the next engine's noise buffer is fresh: draw again
        self._engine_built_for = None
        self._bound = None
        self._fast = None
        self._xmode = None
        self._sampled_pool.clear()
