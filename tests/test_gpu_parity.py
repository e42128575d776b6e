"""GPU parity: the HIP path (through the C ABI) against the golden fixtures
captured from the reference and against the fp64 oracles.

Tolerances (fp32 device arithmetic vs the fp64 reference, BASELINE.json
north_star: "control output within 1e-4 rel-err of the NumPy reference"):
  * u (updated control sequence): max |du| / max(|u|, 1) <= 1e-4
  * S (per-sample cost): relative error <= 5e-5, same argmin
  * trajectories: |dx| <= 1e-4 (1 + |x|)
"""
import math

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import coracle  # noqa: E402
import mppi_oracle as O  # noqa: E402
from conftest import LOOP_FIXTURES, STEP_FIXTURES, ctor_kwargs, load_loop, load_step, record  # noqa: E402

U_TOL = 1e-4
S_TOL = 5e-5

RUNPY = dict(param_exploration=0.0, param_lambda=100.0, param_alpha=0.98, sigma=np.eye(2) * 20.0,
             stage_cost_weight=np.array([0.5, 0.5, 5.0, 5.0]),
             terminal_cost_weight=np.array([5.0, 5.0, 50.0, 50.0]))
X0 = np.array([1.152198236517471885e00, -1.266101672070702344e00, 0.0, 0.0])


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


def _ctrl(g, paths, **kw):
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    c = MPPIControllerForPathTracking(ref_path=paths[str(g["path"])], verbose=False, **ctor_kwargs(g), **kw)
    c.prev_waypoints_idx = int(g["prev_idx"])
    c.u_prev = g["u_prev"].copy()
    return c


def _urel(a, b):
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def _engine(K, T, lps=0, K_total=None, k_offset=0, **over):
    from mppi_robotarm_amd.engine import RolloutEngine
    from mppi_robotarm_amd.params import ArmParams
    kw = dict(RUNPY)
    kw.update(over)
    return RolloutEngine(K, T, 0.006, kw["param_lambda"], kw["param_alpha"], kw["sigma"],
                         kw["stage_cost_weight"], kw["terminal_cost_weight"], kw["param_exploration"],
                         ArmParams(), K_total=K_total, k_offset=k_offset, device=0, lanes_per_sample=lps)


@pytest.mark.parametrize("name", STEP_FIXTURES)
def test_step_matches_reference(name, paths):
    g = load_step(name)
    c = _ctrl(g, paths)
    c.keep_costs = True
    eps = g["eps"].astype(np.float64)
    c._calc_epsilon = lambda *a, **k: eps
    u_prev = c.u_prev
    u0, u_seq, opt, samp = c.calc_control_input(g["x0"])
    S = c.last_S
    assert int(np.argmin(S)) == int(np.argmin(g["S"]))
    assert float(np.max(np.abs(S - g["S"]) / np.abs(g["S"]))) < S_TOL
    assert _urel(u_seq, g["u_seq"]) < U_TOL
    assert _urel(u0, g["u0"]) < U_TOL
    assert u_seq is u_prev and np.shares_memory(u0, u_prev)       # control.py:70,148-152
    assert c.prev_waypoints_idx == int(g["prev_idx_after"])
    np.testing.assert_allclose(opt, g["optimal_traj"], rtol=1e-4, atol=1e-4)
    if "sampled_traj" in g:
        np.testing.assert_allclose(samp, g["sampled_traj"], rtol=1e-4, atol=1e-4)
    else:
        assert not np.any(samp)
    c.close()


@pytest.mark.parametrize("name", ["c1_circle_k128_t20", "runpy_k100_t30", "sigma_k128_t20"])
def test_dropin_consumes_reference_rng_stream(name, paths):
    """np.random.seed(s) + calc_control_input draws the same noise the reference drew."""
    g = load_step(name)
    c = _ctrl(g, paths)
    np.random.seed(int(g["seed"]))
    u0, u_seq, opt, _ = c.calc_control_input(g["x0"])
    assert _urel(u_seq, g["u_seq"]) < U_TOL
    c.close()


@pytest.mark.parametrize("name", LOOP_FIXTURES)
def test_closed_loop_ticks(name, paths):
    """Each tick of run.py's loop from the reference's own state / u_prev / index."""
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    g = load_loop(name)
    T, K = int(g["T"]), int(g["K"])
    c = MPPIControllerForPathTracking(delta_t=0.006, ref_path=paths["xydq_circle"], horizon_step_T=T,
                                      number_of_samples_K=K, verbose=False, visualize_optimal_traj=False,
                                      **RUNPY)
    u_prev = np.array([[10.0, -2.0]] * T)
    prev = 0
    for i in range(int(g["ticks"])):
        c.u_prev = u_prev.copy()
        c.prev_waypoints_idx = prev
        eps = g["eps"][i].astype(np.float64)
        c._calc_epsilon = lambda *a, e=eps, **k: e
        u, u_seq, _, _ = c.calc_control_input(g["states"][i])
        assert _urel(u_seq, g["u_seq"][i]) < U_TOL, i
        assert c.prev_waypoints_idx == int(g["prev_idx"][i])
        u_prev, prev = g["u_seq"][i].copy(), int(g["prev_idx"][i])
    c.close()


def _window(paths, prev=0):
    return paths["xydq_circle"][prev:prev + 30]


@pytest.mark.parametrize("K,T,lam,lps", [(65536, 64, 100.0, 0), (65536, 64, 3.0e6, 0), (65536, 64, 100.0, 2),
                                         (4096, 32, 100.0, 0), (4096, 32, 100.0, 8), (4096, 32, 100.0, 16), (3000, 7, 100.0, 1), (20000, 128, 1.0e6, 0),
                                         (262144, 16, 100.0, 0), (262144, 16, 3.0e6, 0)])
def test_large_rollout_against_c_oracle(K, T, lam, lps, paths):
    """Full-size S and the full weighted noise vs the C fp64 oracle (one-hot and
    dense weights, every lanes-per-sample variant, T up to the 128 limit; the
    262144-sample grid (512 workgroups) takes the counter hand-off with acquire)."""
    eng = _engine(K, T, lps=lps, param_lambda=lam)
    assert eng.handoff == ("poll" if eng.blocks <= torch.cuda.get_device_properties(0).multi_processor_count
                           else "counter")
    win = _window(paths)
    u = np.array([[10.0, -2.0]] * T) + np.random.default_rng(1).normal(0, 0.5, (T, 2))
    eng.set_step_inputs(X0, win, u)
    noise = eng.philox_noise(42, 3)
    S_dev = torch.empty(K, dtype=torch.float64, device="cuda")
    eng.rollout(noise, S_out=S_dev)
    w_eps = eng.weighted_noise()
    S = S_dev.cpu().numpy()
    eps_tk = noise.cpu().numpy()
    ref_S = coracle.rollout_costs(X0, u, eps_tk, win, 0.006, lam, 0.98, np.eye(2) * 20.0,
                                  RUNPY["stage_cost_weight"], RUNPY["terminal_cost_weight"], O.ArmParams(),
                                  layout="TK")
    rel = np.abs(S - ref_S) / np.abs(ref_S)
    assert float(np.max(rel)) < S_TOL
    assert int(np.argmin(S)) == int(np.argmin(ref_S))
    _, ref_weps = coracle.weighted_noise(ref_S, eps_tk, lam, layout="TK")
    assert _urel(w_eps, ref_weps) < U_TOL
    eng.close()


def _fused_steps(eng, paths, noises, T):
    """Device closed loop: fused rollout+update launches, one per noise buffer."""
    eng.set_step_inputs(X0, _window(paths, 3), np.array([[10.0, -2.0]] * T))
    out = []
    for nz in noises:
        eng.rollout(nz, fused_update=True)
        out.append((eng.weighted_noise(), eng.nominal()))
    return out


@pytest.mark.parametrize("lam", [100.0, 3.0e6])
def test_handoff_forms_are_bit_identical(lam, paths, monkeypatch):
    """Granule polling and arrival counters merge the same rows in the same order:
    same bits, over consecutive launches (the granule epoch advances per launch)."""
    K, T = 65536, 64
    runs = {}
    for form in ("poll", "counter"):
        if form == "counter":
            monkeypatch.setenv("MPPI_HANDOFF", "counter")
        eng = _engine(K, T, param_lambda=lam)
        assert eng.handoff == form
        noises = [eng.philox_noise(11, s) for s in range(4)]
        runs[form] = _fused_steps(eng, paths, noises, T)
        eng.synchronize()
        eng.close()
    for (wp, up), (wc, uc) in zip(runs["poll"], runs["counter"]):
        assert np.array_equal(wp, wc)
        assert np.array_equal(up, uc)


def test_graph_replay_matches_eager(paths):
    """HIP-graph replay of fused launches (frozen kernel arguments; the granule
    epoch lives in device memory) == the same launches issued eagerly.  An even
    number of launches brings the ping-pong step block back to where
    set_step_inputs writes the nominal."""
    K, T, n = 65536, 64, 4
    eng = _engine(K, T)
    assert eng.handoff == "poll"
    noises = [eng.philox_noise(5, s) for s in range(n)]
    eager = _fused_steps(eng, paths, noises, T)
    eng.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=s):
        for nz in noises:
            eng.rollout(nz, fused_update=True)
    torch.cuda.current_stream().wait_stream(s)
    for rep in range(3):   # every replay advances the epoch with the same kernel arguments
        eng.set_step_inputs(X0, _window(paths, 3), np.array([[10.0, -2.0]] * T))
        eng.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(eng.weighted_noise(), eager[-1][0]), rep
        assert np.array_equal(eng.nominal(), eager[-1][1]), rep
    eng.close()


@pytest.mark.parametrize("lam", [100.0, 1.0e7])
def test_deterministic_and_lanes_per_sample_invariant(lam, paths):
    """S is bit-identical for every lanes-per-sample split (the split search is
    exact).  w_eps: bit-identical with few weighted samples; with dense weights
    the workgroups (32-256 samples each) sum in another order, so 1e-10."""
    K, T = 20000, 48
    outs = []
    for lps in (1, 2, 4, 8, 16, 2):
        eng = _engine(K, T, lps=lps, param_lambda=lam)
        eng.set_step_inputs(X0, _window(paths, 5), np.array([[10.0, -2.0]] * T))
        noise = eng.philox_noise(7, 0)
        S_dev = torch.empty(K, dtype=torch.float64, device="cuda")
        eng.rollout(noise, S_out=S_dev)
        outs.append((S_dev.cpu().numpy(), eng.weighted_noise()))
        eng.close()
    for S, w in outs[1:]:
        assert np.array_equal(S, outs[0][0])     # the split search is exact: same bits
        if lam == 100.0:
            assert np.array_equal(w, outs[0][1])
        else:
            np.testing.assert_allclose(w, outs[0][1], rtol=1e-10, atol=1e-13)
    assert np.array_equal(outs[1][1], outs[5][1])   # same build, same split: deterministic


def test_shard_invariance_and_merge(paths):
    """G virtual shards on one device + device merge == unsharded."""
    K, T, G = 12288, 32, 4
    u = np.array([[10.0, -2.0]] * T)
    kw = dict(param_lambda=3.0e6, param_alpha=0.95)          # non-degenerate weights
    full = _engine(K, T, **kw)
    full.set_step_inputs(X0, _window(paths), u)
    noise = full.philox_noise(99, 1)
    full.rollout(noise)
    w_full = full.weighted_noise()
    parts = torch.empty(G * full.partial_len, dtype=torch.float64, device="cuda")
    Kl = K // G
    engs = []
    for g in range(G):
        e = _engine(Kl, T, K_total=K, k_offset=g * Kl, **kw)
        e.set_step_inputs(X0, _window(paths), u)
        nz = e.philox_noise(99, 1)
        assert torch.equal(nz, noise[:, g * Kl:(g + 1) * Kl])   # Philox slice == unsharded draw
        e.rollout(nz, partial_out=parts[g * e.partial_len:(g + 1) * e.partial_len])
        engs.append(e)
    engs[0].merge(parts, G)
    w_sh = engs[0].weighted_noise()
    np.testing.assert_allclose(w_sh, w_full, rtol=1e-10, atol=1e-12)
    ess = None  # weights must really be spread for this test to mean something
    S_dev = torch.empty(K, dtype=torch.float64, device="cuda")
    full.rollout(noise, S_out=S_dev)
    S = S_dev.cpu().numpy()
    w = np.exp(-(S - S.min()) / 3.0e6)
    ess = w.sum() ** 2 / (w ** 2).sum()
    assert ess > 10
    for e in engs + [full]:
        e.close()


@pytest.mark.parametrize("T,lam", [(5, 100.0), (6, 100.0), (7, 1.0e4), (8, 100.0), (9, 1.0e4), (10, 100.0),
                                   (12, 1.0e4), (15, 100.0), (16, 1.0e4), (40, 100.0)])
def test_fused_device_update_matches_host_update(T, lam, paths):
    """The fused update's median (a 29-comparator network over the reflected
    window [t-5, t+4]) and u += w_eps + shift (control.py:120-149) against
    scipy.ndimage.median_filter(size=10, mode='reflect') and the fp64 add on the
    host: bit-equal, including the short horizons T = 5..15 where the 10-wide
    window reflects at both ends for most rows (control.py:319-327)."""
    from scipy.ndimage import median_filter
    K = 8192
    eng = _engine(K, T, param_lambda=lam)
    u = np.array([[10.0, -2.0]] * T) + np.random.default_rng(3).normal(0, 0.3, (T, 2))
    eng.set_step_inputs(X0, _window(paths), u)
    for step in range(3):
        noise = eng.philox_noise(5, step)
        eng.rollout(noise, fused_update=True)
        w = eng.weighted_noise()
        filt = np.stack([median_filter(w[:, d], size=10, mode="reflect") for d in range(2)], 1)
        un = u + filt
        expect = np.concatenate([un[1:], un[-1:]], 0)
        got = eng.nominal()
        np.testing.assert_array_equal(got, expect)
        u = got
    eng.close()


def test_exploration_split_across_shards(paths):
    K, T = 1000, 16
    kw = dict(param_exploration=0.37)
    full = _engine(K, T, **kw)
    full.set_step_inputs(X0, _window(paths), np.array([[10.0, -2.0]] * T))
    noise = full.philox_noise(1, 0)
    S_full = torch.empty(K, dtype=torch.float64, device="cuda")
    full.rollout(noise, S_out=S_full)
    ref = coracle.rollout_costs(X0, np.array([[10.0, -2.0]] * T), noise.cpu().numpy(), _window(paths), 0.006,
                                100.0, 0.98, np.eye(2) * 20.0, RUNPY["stage_cost_weight"],
                                RUNPY["terminal_cost_weight"], O.ArmParams(),
                                k_exploit=math.ceil(0.63 * K), layout="TK")
    assert float(np.max(np.abs(S_full.cpu().numpy() - ref) / np.abs(ref))) < S_TOL
    sh = _engine(400, T, K_total=K, k_offset=600, **kw)
    sh.set_step_inputs(X0, _window(paths), np.array([[10.0, -2.0]] * T))
    nz = sh.philox_noise(1, 0)
    S_sh = torch.empty(400, dtype=torch.float64, device="cuda")
    sh.rollout(nz, S_out=S_sh)
    assert np.array_equal(S_sh.cpu().numpy(), S_full.cpu().numpy()[600:])
    full.close()
    sh.close()


def test_philox_noise_statistics():
    K, T = 65536, 64
    sig = np.array([[20.0, 6.0], [6.0, 12.0]])
    eng = _engine(K, T, sigma=sig)
    z = eng.philox_noise(11, 0).double().reshape(-1, 2).cpu().numpy()
    cov = np.cov(z.T)
    np.testing.assert_allclose(z.mean(0), 0.0, atol=0.02)
    np.testing.assert_allclose(cov, sig, rtol=0.01, atol=0.03)
    z2 = eng.philox_noise(11, 1).cpu().numpy()
    assert not np.array_equal(z2.reshape(-1, 2), z.astype(np.float32))
    eng.close()


def test_window_truncated_at_path_end(paths):
    g = load_step("end_k64_t16")
    ref = paths["xydq_circle"]
    prev = int(g["prev_idx_after"])
    win = ref[prev:prev + 30]
    assert win.shape[0] < 30
    eng = _engine(int(g["K"]), int(g["T"]))
    eng.set_step_inputs(g["x0"], win, g["u_prev"])
    noise = eng.upload_noise(g["eps"])
    S_dev = torch.empty(int(g["K"]), dtype=torch.float64, device="cuda")
    eng.rollout(noise, S_out=S_dev)
    S = S_dev.cpu().numpy()
    assert float(np.max(np.abs(S - g["S"]) / g["S"])) < S_TOL
    eng.close()


def test_error_paths(paths):
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    with pytest.raises(np.linalg.LinAlgError):
        _engine(64, 8, sigma=np.array([[10.0, 10.0], [100.0, 100.0]]))
    with pytest.raises(ValueError):
        _engine(64, 129)
    eng = _engine(64, 8)
    with pytest.raises(ValueError):
        eng.rollout(torch.zeros((8, 63, 2), device="cuda"))
    with pytest.raises(ValueError):
        eng.set_step_inputs(X0, np.zeros((31, 4)))
    eng.close()
    # default (singular) sigma raises LinAlgError at the reference's point, after the draw
    c = MPPIControllerForPathTracking(delta_t=0.006, ref_path=paths["xydq_circle"], horizon_step_T=8,
                                      number_of_samples_K=4, verbose=False)
    with pytest.raises(np.linalg.LinAlgError):
        with np.errstate(all="ignore"):
            import warnings
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                c.calc_control_input(X0)


def test_free_running_closed_loop_tracks_reference(paths):
    """run.py's loop (harness) with the drop-in, free-running: at EVERY tick the fp64
    oracle, given the same input state, u_prev, window index and noise draw, returns
    the same control (U_TOL); the trajectory stays on the reference's recorded one.

    A free-running loop amplifies rounding through the plant (the input states drift
    apart tick by tick), so the lockstep oracle carries the parity claim and the
    recorded reference states only a loose tracking bound."""
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    from mppi_robotarm_amd.harness import run_closed_loop
    from mppi_robotarm_amd.params import runpy_config
    g = load_loop("k64_t20")
    T, K = int(g["T"]), int(g["K"])
    kw = dict(runpy_config(), number_of_samples_K=K, horizon_step_T=T, visualze_sampled_trajs=False)
    ctrl = MPPIControllerForPathTracking(ref_path=paths["xydq_circle"], verbose=False, **kw)
    oc = O.OracleController(ref_path=paths["xydq_circle"], **{k: v for k, v in kw.items()
                                                             if k != "visualze_sampled_trajs"})
    oc.visualize_optimal_traj = False
    draws = []
    draw = ctrl._calc_epsilon
    ctrl._calc_epsilon = lambda *a, **k: draws.append(draw(*a, **k)) or draws[-1]
    step = ctrl.calc_control_input
    worst = [0.0]

    def lockstep(observed_x):
        x = np.array(observed_x, dtype=np.float64)
        oc.u_prev = ctrl.u_prev.copy()
        oc.prev_waypoints_idx = ctrl.prev_waypoints_idx
        out = step(observed_x=observed_x)
        _, ou_seq, _, _ = oc.calc_control_input(x, epsilon=draws[-1])
        worst[0] = max(worst[0], _urel(out[1], ou_seq))
        assert _urel(out[1], ou_seq) < U_TOL, len(draws)
        return out

    ctrl.calc_control_input = lockstep
    np.random.seed(int(g["seed"]))
    seen = []
    run_closed_loop(paths["xydq_circle"], ticks=int(g["ticks"]), controller=ctrl,
                    on_tick=lambda k, s, u: seen.append(np.array(s)))
    assert len(draws) == int(g["ticks"]) and worst[0] < U_TOL
    ref = np.vstack([g["states"][1:], g["final_state"][None]])
    # loose: the fp64 oracle itself, free-running on unrounded draws, ends 8e-3 away
    # from the reference's recorded states (fp32-rounded draws) after these 25 ticks
    np.testing.assert_allclose(np.array(seen), ref, atol=5e-2)
    ctrl.close()


@pytest.mark.parametrize("name", ["runpy_k100_t30", "dense_k256_t24", "end_k64_t16", "expl_k128_t20"])
def test_fused_dropin_equals_host_update_path(name, paths):
    """The default drop-in (update inside the launch, optimal trajectory from the
    update, one read-back) against host_update=True (scipy median on the host, as
    the reference): identical u, u0 aliasing, trajectories and S."""
    g = load_step(name)
    eps = g["eps"].astype(np.float64)
    outs = []
    for host in (False, True):
        c = _ctrl(g, paths, host_update=host)
        c.keep_costs = True
        c._calc_epsilon = lambda *a, **k: eps
        u_prev = c.u_prev
        u0, u_seq, opt, samp = c.calc_control_input(g["x0"])
        assert u_seq is u_prev and np.shares_memory(u0, u_prev)
        outs.append((u_seq.copy(), float(u0[0]), opt.copy(), samp.copy(), c.last_S.copy()))
        c.close()
    (ua, u0a, oa, sa, Sa), (ub, u0b, ob, sb, Sb) = outs
    assert np.array_equal(ua, ub) and u0a == u0b
    assert np.array_equal(oa, ob) and np.array_equal(sa, sb) and np.array_equal(Sa, Sb)


def test_fused_dropin_device_noise_loop_equals_host_update(paths):
    """A closed loop with device noise (next step's noise drawn at the end of each
    call): the fused path and the host-update path give the same trajectory."""
    from mppi_robotarm_amd.harness import run_closed_loop
    recs = []
    for host in (False, True):
        rec = run_closed_loop(paths["xydq_circle"][:, :4], ticks=12, number_of_samples_K=4096, horizon_step_T=32,
                              noise="device", seed=5, verbose=False, visualze_sampled_trajs=False, device=0,
                              host_update=host)
        recs.append((rec["u"].copy(), rec["q"].copy()))
        rec["controller"].close()
    assert np.array_equal(recs[0][0], recs[1][0]) and np.array_equal(recs[0][1], recs[1][1])


@pytest.mark.parametrize("K,T,lam", [(1, 1, 100.0), (2, 2, 100.0), (63, 3, 100.0), (65, 4, 3.0e6), (257, 1, 3.0e6),
                                     (1000, 5, 100.0)])
def test_tiny_and_ragged_sizes_against_c_oracle(K, T, lam, paths):
    """Edge sizes: one sample, one step, K not a multiple of the wave or workgroup (partial waves, idle
    lanes), the shortest horizons; S and the weighted noise against the C fp64 oracle."""
    eng = _engine(K, T, param_lambda=lam)
    win = _window(paths)
    u = np.array([[10.0, -2.0]] * T) + np.random.default_rng(K + T).normal(0, 0.5, (T, 2))
    eng.set_step_inputs(X0, win, u)
    noise = eng.philox_noise(7, 1)
    S_dev = torch.empty(K, dtype=torch.float64, device="cuda")
    eng.rollout(noise, S_out=S_dev)
    w_eps = eng.weighted_noise()
    S = S_dev.cpu().numpy()
    eps_tk = noise.cpu().numpy()
    ref_S = coracle.rollout_costs(X0, u, eps_tk, win, 0.006, lam, 0.98, np.eye(2) * 20.0,
                                  RUNPY["stage_cost_weight"], RUNPY["terminal_cost_weight"], O.ArmParams(),
                                  layout="TK")
    assert float(np.max(np.abs(S - ref_S) / np.abs(ref_S))) < S_TOL
    assert int(np.argmin(S)) == int(np.argmin(ref_S))
    _, ref_weps = coracle.weighted_noise(ref_S, eps_tk, lam, layout="TK")
    assert _urel(w_eps, ref_weps) < U_TOL
    eng.close()


@pytest.mark.parametrize("K,T", [(1, 1), (5, 2), (64, 3), (100, 4), (130, 5)])
def test_dropin_short_horizons_match_oracle_controller(K, T, paths):
    """The drop-in at horizons below the median window (T < 5: host update through SciPy's reflect
    padding; T = 5: the fused device update) against the fp64 oracle controller, three closed-loop ticks
    on the same NumPy noise, including the aliasing of the returns."""
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    kw = dict(delta_t=0.006, ref_path=paths["xydq_circle"], horizon_step_T=T, number_of_samples_K=K,
              visualize_optimal_traj=True, **RUNPY)
    c = MPPIControllerForPathTracking(verbose=False, **kw)
    o = O.OracleController(**kw)
    x = X0.copy()
    rng = np.random.default_rng(K * 10 + T)
    for tick in range(3):
        eps = rng.multivariate_normal(np.zeros(2), RUNPY["sigma"], (K, T)).astype(np.float32).astype(np.float64)
        c._calc_epsilon = lambda *a, e=eps, **k: e
        u_prev = c.u_prev
        u0, u_seq, opt, _ = c.calc_control_input(x)
        r0, r_seq, r_opt, _ = o.calc_control_input(x, epsilon=eps)
        assert _urel(u_seq, r_seq) < U_TOL, tick
        assert _urel(np.asarray(u0), np.asarray(r0)) < U_TOL, tick
        assert u_seq is u_prev and np.shares_memory(u0, u_prev)
        assert c.prev_waypoints_idx == o.prev_waypoints_idx
        np.testing.assert_allclose(opt, r_opt, rtol=1e-4, atol=1e-4)
        x = r_opt[-1].copy()
    c.close()


@pytest.mark.parametrize("lam", [100.0, 3.0e6])
def test_config4_eight_virtual_shards(lam, paths, monkeypatch):
    """BASELINE config 4 at its real geometry on one device: K = 524288, T = 64,
    sharded as 8 x 65536 (the per-GPU shard of the 8-GPU run, control.py:91-118
    restricted to a K slice).  Each shard draws its Philox slice (== the slice of
    the unsharded draw), rolls out into a partial row, and the 8 rows are merged
    with the fused update; against (i) one unsharded K = 524288 launch (1e-10)
    and (ii) the C fp64 oracle at full size (S <= 5e-5 rel, same argmin,
    w_eps <= 1e-4).  lam = 3e6 spreads the weights over many shards.

    The unsharded launch is held to the shards' 256-thread workgroups, so the
    two runs partition the samples the same way and only the fp64 merge order
    differs (the weights are fp64 relative to each workgroup's minimum; another
    partition changes the summation order only, <= 1e-10)."""
    K, T, G = 524288, 64, 8
    Kl = K // G
    u = np.array([[10.0, -2.0]] * T) + np.random.default_rng(4).normal(0, 0.5, (T, 2))
    win = _window(paths)
    monkeypatch.setenv("MPPI_BLOCK", "256")
    full = _engine(K, T, param_lambda=lam)
    monkeypatch.delenv("MPPI_BLOCK")
    assert full.threads == 256
    assert full.handoff == "counter"     # 2048 workgroups: more than one per CU
    full.set_step_inputs(X0, win, u)
    noise = full.philox_noise(2024, 9)
    S_full = torch.empty(K, dtype=torch.float64, device="cuda")
    full.rollout(noise, S_out=S_full)
    w_full = full.weighted_noise()
    full.set_step_inputs(X0, win, u)
    full.rollout(noise, fused_update=True)
    u_full = full.nominal()
    parts = torch.empty(G * (2 + 2 * T), dtype=torch.float64, device="cuda")
    S_sh = torch.empty(K, dtype=torch.float64, device="cuda")
    engs = []
    for g in range(G):
        e = _engine(Kl, T, K_total=K, k_offset=g * Kl, param_lambda=lam)
        assert e.handoff == "poll" and e.lanes_per_sample == 1
        e.set_step_inputs(X0, win, u)
        nz = e.philox_noise(2024, 9)
        assert torch.equal(nz, noise[:, g * Kl:(g + 1) * Kl])   # Philox slice == unsharded draw
        e.rollout(nz, S_out=S_sh[g * Kl:(g + 1) * Kl], partial_out=parts[g * e.partial_len:(g + 1) * e.partial_len])
        engs.append(e)
        del nz
    engs[0].merge(parts, G)
    w_sh = engs[0].weighted_noise()
    engs[0].merge(parts, G, fused_update=True)
    u_sh = engs[0].nominal()
    S_dev = S_sh.cpu().numpy()
    assert np.array_equal(S_dev, S_full.cpu().numpy())          # a shard is an exact slice
    np.testing.assert_allclose(w_sh, w_full, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(u_sh, u_full, rtol=1e-10, atol=1e-12)
    eps_tk = noise.cpu().numpy()
    ref_S = coracle.rollout_costs(X0, u, eps_tk, win, 0.006, lam, 0.98, np.eye(2) * 20.0,
                                  RUNPY["stage_cost_weight"], RUNPY["terminal_cost_weight"], O.ArmParams(),
                                  layout="TK")
    rel = np.abs(S_dev - ref_S) / np.abs(ref_S)
    assert float(np.max(rel)) < S_TOL
    assert int(np.argmin(S_dev)) == int(np.argmin(ref_S))
    _, ref_weps = coracle.weighted_noise(ref_S, eps_tk, lam, layout="TK")
    assert _urel(w_sh, ref_weps) < U_TOL
    if lam > 1e6:   # the weights really are spread over the shards
        w = np.exp(-(ref_S - ref_S.min()) / lam)
        assert w.sum() ** 2 / (w ** 2).sum() > 100
        assert len({int(k) // Kl for k in np.argsort(ref_S)[:64]}) == G
    print(f"config 4 lam={lam}: S max rel-err {float(np.max(rel)):.2e}, w_eps rel-err {_urel(w_sh, ref_weps):.2e}")
    record("config4", lam=lam, S_max_rel_err=float(np.max(rel)), S_p99_rel_err=float(np.percentile(rel, 99)),
           w_eps_rel_err=_urel(w_sh, ref_weps))
    for e in engs + [full]:
        e.close()


def _runpy_ctrl(paths, K=4096, T=32, **kw):
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    return MPPIControllerForPathTracking(delta_t=0.006, horizon_step_T=T, number_of_samples_K=K, verbose=False,
                                         **{"ref_path": paths["xydq_circle"], **RUNPY, **kw})


def test_device_noise_ticks_on_alternating_streams(paths):
    """noise='device' draws the next tick's noise asynchronously after the read-back;
    a caller that issues each tick on a different torch stream must still roll out
    the finished draw (the engine makes the new stream wait for the old one)."""
    ref = _runpy_ctrl(paths, noise="device", seed=5)
    want = [ref.calc_control_input(X0)[1].copy() for _ in range(4)]
    ref.close()
    c = _runpy_ctrl(paths, noise="device", seed=5)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for i in range(4):
        with torch.cuda.stream(streams[i % 2]):
            got = c.calc_control_input(X0)[1].copy()
        assert np.array_equal(got, want[i]), i
    c.close()


def test_close_then_continue_redraws_device_noise(paths):
    """close() drops the engine and its noise buffer; the next call must draw the
    step's noise into the new buffer, not trust the old 'noise ready' mark."""
    a = _runpy_ctrl(paths, noise="device", seed=9)
    a.calc_control_input(X0)
    want = a.calc_control_input(X0)[1].copy()
    a.close()
    b = _runpy_ctrl(paths, noise="device", seed=9)
    b.calc_control_input(X0)
    b.close()
    got = b.calc_control_input(X0)[1].copy()
    assert np.array_equal(got, want)
    b.close()


def test_sigma_and_lambda_reread_per_call(paths):
    """The reference reads self.Sigma (control.py:84,106) and self.param_lambda
    (:112) on every call, with gamma fixed at construction (:45): changing them
    between calls must act on the next step exactly as a controller built with
    the new values (and the constructor's gamma) would."""
    sig2 = np.array([[12.0, 3.0], [3.0, 25.0]])
    c = _runpy_ctrl(paths)
    np.random.seed(1)
    c.calc_control_input(X0)
    c.Sigma = sig2
    c.param_lambda = 40.0
    u_prev, prev = c.u_prev.copy(), c.prev_waypoints_idx
    np.random.seed(2)
    got = c.calc_control_input(X0)[1].copy()
    c.close()
    oc = O.OracleController(delta_t=0.006, ref_path=paths["xydq_circle"], horizon_step_T=32,
                            number_of_samples_K=4096, **{**RUNPY, "sigma": sig2, "param_lambda": 40.0})
    oc.param_gamma = RUNPY["param_lambda"] * (1.0 - RUNPY["param_alpha"])   # gamma as constructed (control.py:45)
    oc.u_prev, oc.prev_waypoints_idx = u_prev, prev
    np.random.seed(2)
    eps = np.random.multivariate_normal(np.zeros(2), sig2, (4096, 32)).astype(np.float32).astype(np.float64)
    want = oc.calc_control_input(X0, epsilon=eps)[1]
    assert _urel(got, want) < U_TOL


@pytest.mark.parametrize("noise", ["numpy", "device"])
def test_sample_count_and_horizon_reread_per_call(noise, paths):
    """self.K and self.T are read on every call (control.py:81-95): changing them between calls (with a
    u_prev of the new horizon) must act on the next step exactly as a controller built with the new values
    would — including a horizon below 5, which takes the host update."""
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    kw = dict(delta_t=0.006, verbose=False, noise=noise, seed=5, device=0, **RUNPY)
    c = MPPIControllerForPathTracking(ref_path=paths["xydq_circle"], horizon_step_T=16, number_of_samples_K=2048, **kw)
    np.random.seed(1)
    c.calc_control_input(X0)
    c.calc_control_input(X0)
    for K, T in ((1000, 12), (3000, 4), (2048, 16)):
        u0 = np.tile([[9.0, -1.5]], (T, 1)) + 0.01 * np.arange(T)[:, None]
        c.K, c.T, c.u_prev = K, T, u0.copy()
        ref = MPPIControllerForPathTracking(ref_path=paths["xydq_circle"], horizon_step_T=T, number_of_samples_K=K,
                                            **kw)
        ref.u_prev, ref.prev_waypoints_idx = u0.copy(), c.prev_waypoints_idx
        if noise == "device":
            ref._step_count = c._step_count             # the same (seed, step) of the device stream
        np.random.seed(7)
        got = c.calc_control_input(X0)
        np.random.seed(7)
        want = ref.calc_control_input(X0)
        assert got[1].shape == (T, 2) and got[3].shape == (K, T, 4)
        assert np.array_equal(got[1], want[1]) and np.array_equal(got[2], want[2]), (K, T)
        assert c.prev_waypoints_idx == ref.prev_waypoints_idx
        ref.close()
    c.close()


def test_bound_tick_equals_general_dropin(paths):
    """The one-call tick (mppi_dropin_tick: native nearest-waypoint update, no
    input copy when u_prev is the nominal the last step published) against the
    general drop-in path on the same device noise, bit for bit: u, the aliasing,
    prev_waypoints_idx and the optimal trajectory, over ticks that move along the
    path, an in-place edit of u_prev and of ref_path between ticks (both must be
    seen), and the end of the path (IndexError at the same index, nothing run)."""
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    base = paths["xydq_circle"][:60].copy()
    kw = dict(delta_t=0.006, horizon_step_T=16, number_of_samples_K=2048, verbose=False, noise="device", seed=3,
              device=0, **RUNPY)
    fast = MPPIControllerForPathTracking(ref_path=base[:, 0:4], **kw)          # strided view, like run.py
    slow = MPPIControllerForPathTracking(ref_path=base[:, 0:4].tolist(), **kw)  # not an ndarray: general path
    slow.ref_path = np.array(slow.ref_path)[:, :4].copy(order="F")             # column-major: no tick either
    assert fast._tick is not None
    x = X0.copy()
    for tick in range(40):
        if tick == 4:
            for c in (fast, slow):
                c.u_prev += 0.25                    # caller edits the nominal in place
        if tick == 6:
            base[10:40, 0] += 1e-3                  # caller edits the path in place (the view sees it)
            slow.ref_path[10:40, 0] += 1e-3
        outs = []
        for c in (fast, slow):
            u_prev = c.u_prev
            try:
                u0, u_seq, opt, samp = c.calc_control_input(x)
            except IndexError:
                outs.append(None)
                continue
            assert u_seq is u_prev and np.shares_memory(u0, u_prev)
            assert samp.shape == (2048, 16, 4) and not samp.any()
            outs.append((u_seq.copy(), opt.copy(), c.prev_waypoints_idx))
        if outs[0] is None or outs[1] is None:
            assert outs[0] is None and outs[1] is None, tick
            assert fast.prev_waypoints_idx == slow.prev_waypoints_idx >= 58
            break
        (ua, oa, ia), (ub, ob, ib) = outs
        assert ia == ib and np.array_equal(ua, ub) and np.array_equal(oa, ob), tick
        x = oa[4].copy()                            # move along the planned trajectory
        if tick >= 8:                               # then jump to the last waypoint (2-link IK, elbow as X0)
            px, py = base[59, 0], base[59, 1]
            q2 = -np.arccos((px * px + py * py - 2.0) / 2.0)
            x = np.array([np.arctan2(py, px) - np.arctan2(np.sin(q2), 1.0 + np.cos(q2)), q2, 0.0, 0.0])
    else:
        raise AssertionError("the path end was never reached")
    assert fast._bound is not None                  # the fast controller really took the tick
    fast.close()
    slow.close()


def test_fast_tick_sees_every_per_call_read(paths):
    """calc_control_input's fast test (the last bound tick's objects, scalars and
    array contents unchanged -> straight to the launch) against a controller that
    runs every check on every call, bit for bit, while the caller edits what the
    reference re-reads per call between ticks: Sigma in place and rebound
    (control.py:84,106), lambda (:112), the stage weights in place (:185), the
    exploration split (:98), the seed (device noise), prev_waypoints_idx and
    ref_path rebound."""
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    base = paths["xydq_circle"][:400].copy()
    kw = dict(delta_t=0.006, horizon_step_T=16, number_of_samples_K=2048, verbose=False, noise="device", seed=3,
              device=0, **RUNPY)
    fast = MPPIControllerForPathTracking(ref_path=base[:, 0:4], **kw)
    full = MPPIControllerForPathTracking(ref_path=base[:, 0:4], **kw)
    for c in (fast, full):
        c.Sigma = np.array(c.Sigma, dtype=np.float64)
        c.stage_cost_weight = np.array(c.stage_cost_weight, dtype=np.float64)
        c.terminal_cost_weight = np.array(c.terminal_cost_weight, dtype=np.float64)
    edits = {
        3: lambda c: c.Sigma.__setitem__((0, 0), c.Sigma[0, 0] * 1.5),
        6: lambda c: setattr(c, "param_lambda", 40.0),
        9: lambda c: c.stage_cost_weight.__setitem__(1, 3.0),
        12: lambda c: setattr(c, "Sigma", np.array([[12.0, 3.0], [3.0, 25.0]])),
        15: lambda c: setattr(c, "param_exploration", 0.25),
        18: lambda c: setattr(c, "seed", 11),
        21: lambda c: setattr(c, "prev_waypoints_idx", c.prev_waypoints_idx + 3),
        24: lambda c: setattr(c, "ref_path", base[:, 0:4].copy()),
    }
    slow_calls = []
    tick_checked = fast._tick
    fast._tick = lambda x: (slow_calls.append(1), tick_checked(x))[1]   # every call but the fast test's
    x = X0.copy()
    n = 27
    for tick in range(n):
        if tick in edits:
            for c in (fast, full):
                edits[tick](c)
        full._fast = None                            # every check, every call
        ua, _, oa, _ = fast.calc_control_input(x)
        ub, _, ob, _ = full.calc_control_input(x)
        assert fast.prev_waypoints_idx == full.prev_waypoints_idx, tick
        assert np.array_equal(fast.u_prev, full.u_prev) and np.array_equal(oa, ob), tick
        x = oa[4].copy()
    assert n - len(slow_calls) >= 8                  # the fast test really passed between the edits
    fast.close()
    full.close()


def test_tick_nearest_waypoint_follows_python_min_on_nan_rows(paths):
    """The native tick's waypoint update (mppi_dropin_tick) takes d.index(min(d))
    like the reference (control.py:212-215) and the host path: a NaN row after
    the nearest one is never chosen, a NaN in the window's first row always is."""
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    base = paths["xydq_circle"][:120].copy()
    c = _runpy_ctrl(paths, K=1024, T=16, noise="device", seed=3, ref_path=base)
    c.calc_control_input(X0)                        # builds the engine (general path)
    host = MPPIControllerForPathTracking(ref_path=base, verbose=False)
    host.prev_waypoints_idx = c.prev_waypoints_idx
    want = host._get_nearest_waypoint(X0[0], X0[1])[0]
    base[want + 1, :2] = np.nan
    c.calc_control_input(X0)
    assert c._bound is not None and c.prev_waypoints_idx == want
    base[want, :2] = np.nan                         # the window's first row
    c.calc_control_input(X0)
    assert c.prev_waypoints_idx == want
    c.close()


def _random_cases(n=24, seed=2024):
    rng = np.random.default_rng(seed)
    cases = []
    for i in range(n):
        K = int(rng.choice([1, 7, 64, 100, 777, 2048, 4096, 5000, 12345, 20000]))
        T = int(rng.integers(1, 129))
        lam = float(10 ** rng.uniform(0, 7))
        lps = int(rng.choice([0, 1, 2, 4, 8]))
        expl = float(rng.choice([0.0, 0.0, 0.1, 0.5]))
        prev = int(rng.integers(0, 200)) if i % 4 else int(rng.integers(0, 4000))
        cases.append((i, K, T, lam, lps, expl, prev))
    return cases


@pytest.mark.parametrize("i,K,T,lam,lps,expl,prev", _random_cases())
def test_random_configs_against_c_oracle(i, K, T, lam, lps, expl, prev, paths):
    """Seeded random sweep (control.py:91-118): K from 1 to 20000, T from 1 to 128, lambda over seven
    decades, every lanes-per-sample split, exploration fractions, windows anywhere on the path
    (truncated ones at its end), a random SPD Sigma and start pose.  S to 5e-5, the argmin (or a
    near-tie at fp32 resolution), the weighted noise to 1e-4 against the C fp64 oracle."""
    rng = np.random.default_rng(1000 + i)
    A = rng.normal(0, 1, (2, 2))
    sigma = A @ A.T + np.eye(2) * rng.uniform(2.0, 20.0)
    path = paths["xydq_circle"]
    prev = min(prev, len(path) - 1)
    win = path[prev:prev + 30]
    x0 = X0 + np.concatenate([rng.normal(0, 0.05, 2), rng.normal(0, 0.5, 2)])
    u = np.array([[10.0, -2.0]] * T) + rng.normal(0, 2.0, (T, 2))
    eng = _engine(K, T, lps=lps, param_lambda=lam, param_exploration=expl, sigma=sigma)
    eng.set_step_inputs(x0, win, u)
    noise = eng.philox_noise(11 + i, i)
    S_dev = torch.empty(K, dtype=torch.float64, device="cuda")
    eng.rollout(noise, S_out=S_dev)
    w_eps = eng.weighted_noise()
    S = S_dev.cpu().numpy()
    eps_tk = noise.cpu().numpy()
    ref_S = coracle.rollout_costs(x0, u, eps_tk, win, 0.006, lam, 0.98, sigma, RUNPY["stage_cost_weight"],
                                  RUNPY["terminal_cost_weight"], O.ArmParams(),
                                  k_exploit=math.ceil((1.0 - expl) * K), layout="TK")
    assert float(np.max(np.abs(S - ref_S) / np.abs(ref_S))) < S_TOL
    j, j_ref = int(np.argmin(S)), int(np.argmin(ref_S))
    assert j == j_ref or abs(ref_S[j] - ref_S[j_ref]) <= 1e-6 * abs(ref_S[j_ref])
    _, ref_weps = coracle.weighted_noise(ref_S, eps_tk, lam, layout="TK")
    assert _urel(w_eps, ref_weps) < U_TOL
    eng.close()


def test_sampled_trajs_arrays_stay_the_callers_across_calls(paths):
    """sampled_traj_list comes from pooled read-back arrays (SampledReadback): every call's array matches the
    reference's (control.py:135-145) and no later call writes into an array the caller still holds, written to
    or viewed; dropped arrays' buffers come back."""
    g = load_step("runpy_k100_t30")
    assert "sampled_traj" in g
    c = _ctrl(g, paths)
    eps = g["eps"].astype(np.float64)
    c._calc_epsilon = lambda *a, **k: eps

    def call():
        c.prev_waypoints_idx = int(g["prev_idx"])
        c.u_prev[:] = g["u_prev"]
        samp = c.calc_control_input(g["x0"])[3]
        np.testing.assert_allclose(samp, g["sampled_traj"], rtol=1e-4, atol=1e-4)
        return samp

    held = [call() for _ in range(5)]            # 3 pooled arrays, then fresh ones
    ref = held[0].copy()
    for i, a in enumerate(held):
        assert a.flags.writeable and a.dtype == np.float64
        assert not any(np.shares_memory(a, b) for b in held[i + 1:])
    held[1][:] = -7.0                            # the caller's to write
    view = held[2][3:, 5]
    del held[2:]
    for _ in range(4):
        a = call()
        assert not np.shares_memory(a, held[0]) and not np.shares_memory(a, held[1])
        assert not np.shares_memory(a, view)
    np.testing.assert_array_equal(held[0], ref)
    assert np.all(held[1] == -7.0)
    np.testing.assert_array_equal(view, ref[3:, 5])
    c.close()
