"""RolloutEngine — Python handle on one device context of the HIP engine.

PyTorch-ROCm is used only to own device memory and streams: noise buffers,
per-sample costs, partials and trajectories are torch tensors whose
``data_ptr()`` crosses the C ABI (include/mppi_rocm.h).  All work is issued on
the torch current stream of the engine's device, so ``torch.cuda.Event``
timing and RCCL collectives order with it naturally.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np
import torch

from . import _native as N
from .params import ArmParams


def _raw_stream(index: int) -> int:
    """Handle of torch's current stream on device `index` without building a Stream object."""
    get = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    return get(index) if get is not None else torch.cuda.current_stream(index).cuda_stream


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _upload_std(eng, noise, z: torch.Tensor, out: torch.Tensor, perm) -> torch.Event:
    """RolloutEngine / ChainEngine.upload_std_noise: rows [k_offset, k_offset + K_local) of the (K, T, du)
    standard normals in the page-locked z, to the device, transformed there, into out (layout `perm` of
    (K_local, T, du))."""
    eng._sync_stream()
    K, T, du = noise.z.shape
    lo, kl = eng.k_offset, eng.K_local
    zz = z[:K * T * du].view(K, T, du)[lo:lo + kl]
    stage = getattr(eng, "_noise_stage", None)
    if stage is None or tuple(stage.shape) != (kl, T, du):
        stage = eng._noise_stage = torch.empty((kl, T, du), dtype=torch.float64, device=eng.device)
    stage.copy_(zz, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(eng.stream)   # the engine's stream (its device need not be the current one)
    key = (noise.src.tobytes(), noise.scale.tobytes(), noise.mean.tobytes())
    if getattr(eng, "_std_key", None) != key:
        eng._std_key = key
        eng._std_t = (torch.from_numpy(noise.src).to(eng.device), torch.from_numpy(noise.scale).to(eng.device),
                      torch.from_numpy(noise.mean).to(eng.device),
                      bool(np.array_equal(noise.src, np.arange(du))))
    src, scale, mean, ident = eng._std_t
    x = stage if ident else stage.index_select(2, src)
    x = torch.mul(x, scale)          # the np.dot with one nonzero per column: exact products
    x.add_(mean)                     # x += mean
    out.copy_(x.permute(*perm))      # transpose + fp64 -> fp32 (round to nearest, as astype)
    return ev


class RolloutEngine:
    """Owns one ``mppi_ctx`` (one device, one shard of samples)."""

    def __init__(self, K_local: int, T: int, delta_t: float, param_lambda: float, param_alpha: float,
                 sigma, stage_cost_weight, terminal_cost_weight, param_exploration: float = 0.0,
                 arm: ArmParams = ArmParams(), K_total: int | None = None, k_offset: int = 0,
                 device: int | torch.device | None = None, lanes_per_sample: int = 0,
                 param_gamma: float | None = None):
        self._lib = N.load()
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", device if isinstance(device, int) else device.index)
        self.K_local, self.T = int(K_local), int(T)
        self.K_total = int(K_total if K_total is not None else K_local)
        self.k_offset = int(k_offset)
        cfg = N.ConfigC()
        cfg.K_local, cfg.T, cfg.K_total, cfg.k_offset = self.K_local, self.T, self.K_total, self.k_offset
        cfg.delta_t = float(delta_t)
        cfg.param_lambda = float(param_lambda)
        cfg.param_alpha = float(param_alpha)
        cfg.param_exploration = float(param_exploration)
        sig = np.asarray(sigma, dtype=np.float64).reshape(2, 2)
        for i, v in enumerate(sig.ravel()):
            cfg.sigma[i] = float(v)
        for i in range(4):
            cfg.stage_cost_weight[i] = float(stage_cost_weight[i])
            cfg.terminal_cost_weight[i] = float(terminal_cost_weight[i])
        for f in ("m1", "m2", "l1", "l2", "lc1", "lc2", "g", "fk_l1", "fk_l2"):
            setattr(cfg.arm, f, float(getattr(arm, f)))
        cfg.lanes_per_sample = int(lanes_per_sample)
        # gamma as given (control.py:45 fixes it at construction); None: lambda (1 - alpha)
        cfg.param_gamma = float("nan") if param_gamma is None else float(param_gamma)
        self.sigma = sig
        self.param_lambda = float(param_lambda)
        with torch.cuda.device(self.device):
            self.stream = torch.cuda.current_stream(self.device)
            ctx = C.c_void_p()
            N.check(self._lib.mppi_ctx_create(C.byref(cfg), self.device.index,
                                              C.c_void_p(self.stream.cuda_stream), C.byref(ctx)),
                    "mppi_ctx_create")
        self._ctx = ctx
        lps, blocks, threads = C.c_int(), C.c_int(), C.c_int()
        N.check(self._lib.mppi_ctx_info(ctx, C.byref(lps), C.byref(blocks), C.byref(threads)), "mppi_ctx_info")
        self.lanes_per_sample, self.blocks, self.threads = lps.value, blocks.value, threads.value
        poll = C.c_int()
        N.check(self._lib.mppi_ctx_handoff(ctx, C.byref(poll)), "mppi_ctx_handoff")
        # in-launch hand-off of the workgroup partials: "poll" (tagged granules) or "counter"
        self.handoff = "poll" if poll.value else "counter"
        self.partial_len = 2 + 2 * self.T
        self._weps = np.zeros((self.T, 2))

    # -- lifetime -----------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_ctx", None):
            self._lib.mppi_ctx_destroy(self._ctx)
            self._ctx = None
        self._noise_stage = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def _sync_stream(self):
        """Follow torch's current stream (it may change between calls).  The new
        stream first waits for the old one: work already queued there (a noise
        draw, a rollout writing a buffer the next call reads) is finished before
        anything issued on the new stream runs."""
        if _raw_stream(self.device.index) == self.stream.cuda_stream:   # the usual case, ~0.3 us
            return
        s = torch.cuda.current_stream(self.device)
        if s.cuda_stream != self.stream.cuda_stream:
            s.wait_stream(self.stream)
            self.stream = s
            N.check(self._lib.mppi_set_stream(self._ctx, C.c_void_p(s.cuda_stream)), "mppi_set_stream")

    # -- buffers ------------------------------------------------------------
    def new_noise(self) -> torch.Tensor:
        """Device noise buffer, layout [T][K_local][2] fp32."""
        return torch.empty((self.T, self.K_local, 2), dtype=torch.float32, device=self.device)

    def new_partial(self) -> torch.Tensor:
        return torch.empty(self.partial_len, dtype=torch.float64, device=self.device)

    def upload_noise(self, eps_kt: np.ndarray, out: torch.Tensor | None = None) -> torch.Tensor:
        """Reference-order noise (K_local, T, 2) -> device [T][K_local][2] fp32."""
        out = self.new_noise() if out is None else out
        # the fp64 draw as it is (one pageable copy, the host array free once it returns), then the transpose
        # and the fp64 -> fp32 rounding (to nearest, as NumPy's astype) in one device copy: the host transpose,
        # conversion and per-call page-locked buffer cost ~70 ms at K = 65536, T = 64
        eps = np.ascontiguousarray(eps_kt, dtype=np.float64)
        stage = getattr(self, "_noise_stage", None)
        if stage is None or tuple(stage.shape) != eps.shape:
            stage = self._noise_stage = torch.empty(eps.shape, dtype=torch.float64, device=self.device)
        stage.copy_(torch.from_numpy(eps))
        out.copy_(stage.permute(1, 0, 2))
        return out

    def upload_std_noise(self, noise, z: torch.Tensor, out: torch.Tensor) -> torch.Event:
        """The reference's draw from its standard normals (hostrng.StdNoise `noise`, whose z lives in the
        page-locked tensor `z`; this shard's K_local rows from k_offset): one DMA, then the transform
        x = z[..., src] * scale + mean as NumPy's (separate fp64 multiply and add: exact, so the values equal
        np.random.multivariate_normal's) and the transpose with the rounding to fp32 (upload_noise).  Returns
        the event after the DMA: z must not be rewritten before it."""
        return _upload_std(self, noise, z, out, (1, 0, 2))

    # -- the hot path -------------------------------------------------------
    def set_step_inputs(self, x0, window, u=None) -> None:
        self._sync_stream()
        x0 = np.ascontiguousarray(np.asarray(x0, dtype=np.float64).ravel()[:4])
        win = np.ascontiguousarray(np.asarray(window, dtype=np.float64)[:, :4])
        if win.ndim != 2 or win.shape[0] < 1 or win.shape[0] > N.MPPI_SEARCH_LEN:
            raise ValueError("window must have 1..30 rows of [x, y, dq1, dq2]")
        uu = None
        if u is not None:
            uu = np.ascontiguousarray(np.asarray(u, dtype=np.float64).reshape(self.T, 2))
        N.check(self._lib.mppi_set_step_inputs(self._ctx, _dptr(x0), _dptr(win), win.shape[0],
                                               _dptr(uu) if uu is not None else None),
                "mppi_set_step_inputs")
        self._keep = (x0, win, uu)  # keep host arrays alive until the async copy ran

    def exchange_handle(self, world: int) -> bytes:
        """Allocate this rank's exchange inbox for `world` ranks; its IPC handle (64 B)."""
        buf = C.create_string_buffer(N.MPPI_IPC_HANDLE_BYTES)
        N.check(self._lib.mppi_exchange_handle(self._ctx, int(world), buf), "mppi_exchange_handle")
        return buf.raw

    def exchange_attach(self, rank: int, world: int, handles) -> None:
        """Map every rank's inbox (handles in rank order); then rollout(..., exchange=True)."""
        blob = b"".join(bytes(h) for h in handles)
        if len(blob) != world * N.MPPI_IPC_HANDLE_BYTES:
            raise ValueError("one 64-byte handle per rank")
        N.check(self._lib.mppi_exchange_attach(self._ctx, int(rank), int(world), C.create_string_buffer(blob, len(blob))),
                "mppi_exchange_attach")
        self.exchange_world = int(world)

    def rollout(self, noise: torch.Tensor, S_out: torch.Tensor | None = None,
                partial_out: torch.Tensor | None = None, fused_update: bool = False, exchange: bool = False,
                host_out: bool = False) -> None:
        """control.py:81-118 for this shard; `exchange`: also exchange and merge the ranks' rows in the launch;
        `host_out` (with fused_update): publish the result to host-mapped memory for wait_outputs()."""
        self._sync_stream()
        self._check_noise(noise)
        if S_out is not None:
            assert S_out.dtype == torch.float64 and S_out.numel() >= self.K_local and S_out.device == self.device
        if partial_out is not None:
            assert partial_out.dtype == torch.float64 and partial_out.numel() >= self.partial_len
        N.check(self._lib.mppi_rollout(self._ctx, C.c_void_p(noise.data_ptr()),
                                       C.c_void_p(S_out.data_ptr()) if S_out is not None else None,
                                       C.c_void_p(partial_out.data_ptr()) if partial_out is not None else None,
                                       (N.MPPI_FLAG_FUSED_UPDATE if fused_update else 0)
                                       | (N.MPPI_FLAG_EXCHANGE if exchange else 0)
                                       | (N.MPPI_FLAG_HOST_OUT if host_out else 0)),
                "mppi_rollout")

    def merge(self, partials: torch.Tensor, n: int, fused_update: bool = False, host_out: bool = False) -> None:
        self._sync_stream()
        assert partials.dtype == torch.float64 and partials.is_contiguous()
        assert partials.numel() >= n * self.partial_len
        N.check(self._lib.mppi_merge_partials(self._ctx, C.c_void_p(partials.data_ptr()), int(n),
                                              (N.MPPI_FLAG_FUSED_UPDATE if fused_update else 0)
                                              | (N.MPPI_FLAG_HOST_OUT if host_out else 0)),
                "mppi_merge_partials")

    def wait_outputs(self, x0=None):
        """After a host_out launch: (shifted nominal (T, 2) fp64, fp64 optimal trajectory (T, 4)
        from x0, or None without x0) — mppi_wait_outputs, no stream synchronise."""
        u_out = np.empty((self.T, 2))
        traj = None
        xp = None
        if x0 is not None:
            x = np.ascontiguousarray(np.asarray(x0, dtype=np.float64).ravel()[:4])
            traj = np.empty((self.T, 4))
            xp = _dptr(x)
        N.check(self._lib.mppi_wait_outputs(self._ctx, xp, _dptr(u_out), _dptr(traj) if traj is not None else None),
                "mppi_wait_outputs")
        return u_out, traj

    def weighted_noise(self) -> np.ndarray:
        """w_eps (T, 2) fp64 of the last rollout / merge (synchronising)."""
        self._sync_stream()
        out = np.zeros((self.T, 2))
        N.check(self._lib.mppi_get_weighted_noise(self._ctx, _dptr(out)), "mppi_get_weighted_noise")
        return out

    def nominal(self) -> np.ndarray:
        self._sync_stream()
        out = np.zeros((self.T, 2))
        N.check(self._lib.mppi_get_nominal(self._ctx, _dptr(out)), "mppi_get_nominal")
        return out

    def trajectories(self, base_u=None, noise: torch.Tensor | None = None, K: int | None = None) -> torch.Tensor:
        """(K, T, 4) fp32 states of the off-by-one re-roll (control.py:129-145)."""
        self._sync_stream()
        K = self.K_local if K is None else int(K)
        out = torch.empty((K, self.T, 4), dtype=torch.float32, device=self.device)
        bu = None
        if base_u is not None:
            bu = np.ascontiguousarray(np.asarray(base_u, dtype=np.float64).reshape(self.T, 2))
        if noise is not None:
            self._check_noise(noise)
        N.check(self._lib.mppi_rollout_traj(self._ctx, _dptr(bu) if bu is not None else None,
                                            C.c_void_p(noise.data_ptr()) if noise is not None else None,
                                            K, C.c_void_p(out.data_ptr())),
                "mppi_rollout_traj")
        self._keep_traj = bu
        return out

    def optimal_traj(self, out: torch.Tensor | None = None) -> torch.Tensor:
        """(T, 4) fp32 optimal trajectory (control.py:129-134) from the controls of the
        last fused update, before their shift (mppi_optimal_traj)."""
        self._sync_stream()
        out = torch.empty((self.T, 4), dtype=torch.float32, device=self.device) if out is None else out
        N.check(self._lib.mppi_optimal_traj(self._ctx, C.c_void_p(out.data_ptr())), "mppi_optimal_traj")
        return out

    def step_outputs(self, traj: torch.Tensor | None = None):
        """One synchronising read-back after a fused step: the shifted nominal (T, 2) fp64
        and, if given, the (T, 4) fp32 trajectory tensor as a host array (else None)."""
        self._sync_stream()
        u = np.zeros((self.T, 2))
        tr = np.zeros((self.T, 4), dtype=np.float32) if traj is not None else None
        N.check(self._lib.mppi_get_step_outputs(self._ctx, _dptr(u),
                                                C.c_void_p(traj.data_ptr()) if traj is not None else None,
                                                tr.ctypes.data_as(C.c_void_p) if tr is not None else None),
                "mppi_get_step_outputs")
        return u, tr

    def step_dropin(self, x0, window, u, noise: torch.Tensor, S_out: torch.Tensor | None = None,
                    next_noise: torch.Tensor | None = None, seed: int = 0, next_step: int = 0,
                    want_traj: bool = True):
        """The single-device control step in one native call (mppi_step_dropin):
        stage inputs, fused rollout + update, wait on the host-mapped result, host
        fp64 optimal trajectory, then queue the next step's noise into next_noise.
        Returns (shifted nominal (T, 2) fp64 — a buffer reused by the next call —,
        optimal trajectory (T, 4) fp64 or None)."""
        self._sync_stream()
        x = np.ascontiguousarray(x0, dtype=np.float64)
        if x.shape != (4,):
            x = np.ascontiguousarray(x.ravel()[:4])
        win = window
        if not (isinstance(win, np.ndarray) and win.dtype == np.float64 and win.ndim == 2 and win.shape[1] == 4
                and win.flags.c_contiguous):
            win = np.ascontiguousarray(np.asarray(window, dtype=np.float64)[:, :4])
        if not 1 <= win.shape[0] <= N.MPPI_SEARCH_LEN:
            raise ValueError("window must have 1..30 rows of [x, y, dq1, dq2]")
        uu = None if u is None else np.ascontiguousarray(u, dtype=np.float64)
        if uu is not None and uu.shape != (self.T, 2):
            raise ValueError(f"u must be ({self.T}, 2)")
        if noise.data_ptr() != getattr(self, "_checked_noise", 0):
            self._check_noise(noise)
            self._checked_noise = noise.data_ptr()
        if getattr(self, "_u_out", None) is None:
            self._u_out = np.empty((self.T, 2))
        traj = np.empty((self.T, 4)) if want_traj else None
        N.check(self._lib.mppi_step_dropin(
            self._ctx, x.ctypes.data, win.ctypes.data, win.shape[0], uu.ctypes.data if uu is not None else None,
            noise.data_ptr(), S_out.data_ptr() if S_out is not None else None,
            next_noise.data_ptr() if next_noise is not None else None, seed & 0xFFFFFFFFFFFFFFFF,
            next_step & 0xFFFFFFFFFFFFFFFF,
            self._u_out.ctypes.data, traj.ctypes.data if traj is not None else None), "mppi_step_dropin")
        return self._u_out, traj

    def dropin_bind(self, path: np.ndarray, fk_l1: float, fk_l2: float, x_buf: np.ndarray, idx_buf: np.ndarray,
                    u: np.ndarray, traj_buf: np.ndarray | None, noise: torch.Tensor,
                    next_noise: torch.Tensor | None, S_out: torch.Tensor | None, seed: int) -> None:
        """Bind the host buffers of dropin_tick (mppi_dropin_bind).  path: fp64 (rows, >= 4)
        with unit column stride (any row stride: run.py's ref_path[:, 0:4] is a view); x_buf: fp64 (4,); idx_buf: int64 (2,); u: C-contiguous fp64 (T, 2),
        updated in place; traj_buf: fp64 (T, 4) or None.  The arrays must outlive the
        binding (the caller keeps them)."""
        self._check_noise(noise)
        if next_noise is not None:
            self._check_noise(next_noise)
        b = N.DropinBindingC()
        b.path, b.rows, b.stride = path.ctypes.data, path.shape[0], path.strides[0] // 8
        b.fk_l1, b.fk_l2 = float(fk_l1), float(fk_l2)
        b.x0, b.idx, b.u = x_buf.ctypes.data, idx_buf.ctypes.data, u.ctypes.data
        b.traj = traj_buf.ctypes.data if traj_buf is not None else None
        b.noise_dev = noise.data_ptr()
        b.next_noise_dev = next_noise.data_ptr() if next_noise is not None else None
        b.S_dev = S_out.data_ptr() if S_out is not None else None
        b.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        N.check(self._lib.mppi_dropin_bind(self._ctx, C.byref(b)), "mppi_dropin_bind")

    def dropin_tick(self, next_step: int) -> int:
        """One bound drop-in step (mppi_dropin_tick): MPPI_OK, or MPPI_E_PATH_END
        (nothing launched); any other failure raises."""
        self._sync_stream()
        rc = self._lib.mppi_dropin_tick(self._ctx, next_step)
        if rc != N.MPPI_OK and rc != N.MPPI_E_PATH_END:
            N.check(rc, "mppi_dropin_tick")
        return rc

    def dropin_tick_launch(self, next_step: int) -> int:
        """The launch half of dropin_tick (mppi_dropin_tick_launch): MPPI_OK or
        MPPI_E_PATH_END (nothing launched); dropin_tick_wait() must follow an OK."""
        self._sync_stream()
        rc = self._lib.mppi_dropin_tick_launch(self._ctx, next_step)
        if rc != N.MPPI_OK and rc != N.MPPI_E_PATH_END:
            N.check(rc, "mppi_dropin_tick_launch")
        return rc

    def dropin_tick_wait(self) -> None:
        """The wait half (mppi_dropin_tick_wait): u and traj of the binding written."""
        N.check(self._lib.mppi_dropin_tick_wait(self._ctx), "mppi_dropin_tick_wait")

    def dropin_times(self) -> np.ndarray:
        """Diagnostics: phase ends (us) of the last step_dropin (mppi_debug_dropin_times)."""
        out = np.zeros(5)
        N.check(self._lib.mppi_debug_dropin_times(self._ctx, _dptr(out)), "mppi_debug_dropin_times")
        return out

    def optimal_traj_host(self, x0, u_new) -> np.ndarray:
        """(T, 4) fp64 optimal trajectory of control.py:129-134 from the updated, not yet
        shifted controls u_new (T, 2), on the host (mppi_optimal_traj_host)."""
        x = np.ascontiguousarray(np.asarray(x0, dtype=np.float64).ravel()[:4])
        un = np.ascontiguousarray(u_new, dtype=np.float64).reshape(self.T, 2)
        out = np.empty((self.T, 4))
        N.check(self._lib.mppi_optimal_traj_host(self._ctx, _dptr(x), _dptr(un), _dptr(out)), "mppi_optimal_traj_host")
        return out

    def philox_noise(self, seed: int, step: int = 0, out: torch.Tensor | None = None) -> torch.Tensor:
        self._sync_stream()
        out = self.new_noise() if out is None else out
        self._check_noise(out)
        N.check(self._lib.mppi_noise_philox(self._ctx, int(seed) & (2 ** 64 - 1), int(step) & (2 ** 64 - 1),
                                            C.c_void_p(out.data_ptr())), "mppi_noise_philox")
        return out

    def nearest_slots(self, noise: torch.Tensor, K: int | None = None) -> tuple[np.ndarray, np.ndarray]:
        """Tests: the window slot the rollout picks for each of the first K samples at
        every step (_get_nearest_waypoint in _c, control.py:176-180, 205-215), and the
        fp32 end-effector position it searched for -> (slot (K, T) int32, pos (K, T, 2))."""
        self._sync_stream()
        self._check_noise(noise)
        K = self.K_local if K is None else int(K)
        slot = torch.empty((K, self.T), dtype=torch.int32, device=self.device)
        pos = torch.empty((K, self.T, 2), dtype=torch.float32, device=self.device)
        N.check(self._lib.mppi_debug_nearest(self._ctx, C.c_void_p(noise.data_ptr()), K,
                                             C.c_void_p(slot.data_ptr()), C.c_void_p(pos.data_ptr())),
                "mppi_debug_nearest")
        self.synchronize()
        return slot.cpu().numpy(), pos.cpu().numpy()

    def synchronize(self) -> None:
        N.check(self._lib.mppi_sync(self._ctx), "mppi_sync")

    def _check_noise(self, noise: torch.Tensor) -> None:
        if (noise.dtype != torch.float32 or not noise.is_contiguous() or noise.device != self.device
                or tuple(noise.shape) != (self.T, self.K_local, 2)):
            raise ValueError(f"noise must be a contiguous fp32 {(self.T, self.K_local, 2)} tensor on {self.device}")


def readback_workers() -> int:
    """Host threads of a HostReadback: MPPI_READBACK_WORKERS, else this process's CPUs (OMP_NUM_THREADS when
    set, the GPU box's share), at most 16."""
    import os
    env = os.environ.get("MPPI_READBACK_WORKERS")
    if env:
        return max(1, min(64, int(env)))
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, min(16, n))


class HostReadback:
    """sampled_traj_list's read-back (control.py:135-145, include/mppi_rocm.h mppi_readback_*): the fp32 states
    DMA'd in chunks through a page-locked ring and widened to fp64 (exact) by host threads into the caller's
    array while the later chunks are in flight.  Half the link bytes of a device-side widening, same values."""

    CHUNK = 1 << 20   # floats per chunk (4 MB; the last three 2, 1 and 0.5 MB)
    SLOTS = 8         # ring slots (32 MB page-locked)
    STREAMS = 2       # copy streams: a copy's start-up overlaps the one before it

    def __init__(self, device: torch.device, workers: int | None = None, chunk: int | None = None,
                 slots: int | None = None, streams: int | None = None):
        self._lib = N.load()
        self.device = device
        self.workers = readback_workers() if workers is None else int(workers)
        self.chunk = self.CHUNK if chunk is None else int(chunk)
        self.slots = self.SLOTS if slots is None else int(slots)
        self.streams = self.STREAMS if streams is None else int(streams)
        rb = C.c_void_p()
        with torch.cuda.device(device):
            N.check(self._lib.mppi_readback_create(device.index, self.workers, self.slots, self.chunk, self.streams,
                                                   C.byref(rb)), "mppi_readback_create")
        self._rb = rb

    def run(self, src: torch.Tensor, dst: np.ndarray) -> np.ndarray:
        """dst[...] = src (fp32 device tensor, contiguous) widened to fp64; dst C-contiguous fp64 of the same
        size.  Ordered after the work queued on the device's current stream; returns when dst is written."""
        if not (src.dtype == torch.float32 and src.is_contiguous() and src.device == self.device
                and dst.dtype == np.float64 and dst.flags.c_contiguous and dst.flags.writeable
                and dst.size == src.numel()):
            raise ValueError("HostReadback.run: a contiguous fp32 device tensor into a writable C-contiguous "
                             "fp64 array of the same size")
        N.check(self._lib.mppi_readback_run(self._rb, C.c_void_p(_raw_stream(self.device.index)),
                                            C.c_void_p(src.data_ptr()), C.c_void_p(dst.ctypes.data), src.numel()),
                "mppi_readback_run")
        return dst

    def close(self) -> None:
        if getattr(self, "_rb", None):
            self._lib.mppi_readback_destroy(self._rb)
            self._rb = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


class NpDeviceStream:
    """The reference's noise draw (control.py:154-164: np.random.multivariate_normal on NumPy's legacy global
    RandomState) generated on the device bit for bit (include/mppi_rocm.h mppi_np_*): the MT19937 words, the
    polar method with glibc's log, the Sigma transform (a scaled column permutation, or a 2 x 2 matrix through np.dot's pinned rounding) and the fp32 rounding,
    straight into an engine's noise buffer; the RNG state is read from and written back to np.random, as
    NumPy's own draw leaves it.  One per device; raises RuntimeError at construction when the host pieces it
    needs (hostrng.log_params, hostrng.jump_polys) are unavailable."""

    def __init__(self, device: torch.device):
        from . import hostrng
        self._lib = N.load()
        self.device = device
        params = hostrng.log_params()
        if params is None:
            raise RuntimeError("the device NumPy draw needs libm's log constants (hostrng.log_params)")
        self._params = params
        ctx = C.c_void_p()
        with torch.cuda.device(device):
            N.check(self._lib.mppi_np_ctx_create(device.index, params.ctypes.data, C.byref(ctx)), "mppi_np_ctx_create")
        self._ctx = ctx
        self._jumps = (0, 0)   # (block stride, streams) uploaded
        self._st = N.NpStateC()
        self._st_ref = C.byref(self._st)
        self._key_addr = C.addressof(self._st.key)
        self._P, self._ns = C.c_int(), C.c_int()
        self._P_ref, self._ns_ref = C.byref(self._P), C.byref(self._ns)
        self._targets = {}   # (K, T, du, buffer, slice, strides) -> (plan, NpTargetC, its byref)
        self.draws = 0      # draws queued
        self.retries = 0    # draws that came back MPPI_E_RETRY (the caller then drew on the host)

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            self._lib.mppi_np_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def draw(self, state, shape, plan, out: torch.Tensor, stream, k_offset: int, K_local: int, strides) -> None:
        """Queue the draw of the (K, T, du) standard normals `shape` from `state` (np.random.get_state()) through
        `plan` (hostrng.device_plan: src, scale, mean, psd, mat) into `out` (fp32 device), samples [k_offset, k_offset +
        K_local) at strides (t, k, d); result() returns the state it leaves.  The target struct of a (shape, plan,
        buffer, slice) is built once: the drop-ins alternate two buffers, and this call sits between one draw's
        end and the next one's first kernel."""
        K, T, du = shape
        n = K * T * du
        pos, has_gauss = int(state[2]), int(state[3])
        N.check(self._lib.mppi_np_plan(self._ctx, n, pos, has_gauss, self._P_ref, self._ns_ref), "mppi_np_plan")
        P, ns = self._P.value, self._ns.value
        if self._jumps[0] != P or self._jumps[1] < ns:
            from . import hostrng
            polys = hostrng.jump_polys(P, ns)
            if polys is None:
                raise RuntimeError("MT19937 jump polynomials unavailable")
            polys = np.ascontiguousarray(polys)
            N.check(self._lib.mppi_np_set_jumps(self._ctx, P, ns, polys.ctypes.data if polys.size else None,
                                                N.NP_POLY_WORDS), "mppi_np_set_jumps")
            self._jumps = (P, ns)
        st = self._st
        key = state[1]
        if not (isinstance(key, np.ndarray) and key.dtype == np.uint32 and key.flags.c_contiguous and key.size == 624):
            key = np.ascontiguousarray(key, dtype=np.uint32)
        C.memmove(self._key_addr, key.ctypes.data, 624 * 4)
        st.pos, st.has_gauss, st.gauss = pos, has_gauss, float(state[4])
        ck = (K, T, du, out.data_ptr(), int(k_offset), int(K_local), tuple(int(x) for x in strides))
        hit = self._targets.get(ck)
        if hit is None or hit[0] is not plan:
            t = N.NpTargetC()
            t.out_dev = out.data_ptr()
            t.K, t.T, t.du, t.k_offset, t.K_local = K, T, du, int(k_offset), int(K_local)
            t.stride_t, t.stride_k, t.stride_d = ck[6]
            src, scale, mean = plan[:3]
            for d in range(du):
                t.src[d], t.scale[d], t.mean[d] = int(src[d]), float(scale[d]), float(mean[d])
            mat = plan[4] if len(plan) > 4 else None   # hostrng.device_plan: a general 2 x 2 transform
            t.dot2 = 0 if mat is None else 1
            if mat is not None:
                for i, v in enumerate(np.asarray(mat, dtype=np.float64).ravel()):
                    t.mat[i] = float(v)
            if len(self._targets) >= 8:
                self._targets.clear()
            hit = (plan, t, C.byref(t))
            self._targets[ck] = hit
        N.check(self._lib.mppi_np_draw(self._ctx, C.c_void_p(stream), self._st_ref, n, hit[2]), "mppi_np_draw")
        self.draws += 1

    def result(self):
        """The state the last draw leaves, as np.random.get_state()'s tuple (waits for the draw), or None when
        the draw could not complete (the output incomplete: draw it on the host)."""
        st = self._st
        rc = self._lib.mppi_np_draw_result(self._ctx, C.byref(st))
        if rc == N.MPPI_E_RETRY:
            self.retries += 1
            return None   # too few accepted attempts or a look-back that gave up: np.random untouched
        N.check(rc, "mppi_np_draw_result")
        key = np.frombuffer(st.key, dtype=np.uint32).copy()
        return ("MT19937", key, st.pos, st.has_gauss, st.gauss)


def exploit_count(param_exploration: float, K: int) -> int:
    """Number of samples with ``k < (1 - expl) * K`` (control.py:98)."""
    thr = (1.0 - param_exploration) * K
    return 0 if thr <= 0 else min(K, int(math.ceil(thr)))
