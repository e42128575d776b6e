"""GPU: the n-link chain engine (BASELINE config 5) through the C ABI.

Parity anchors:
  * n = 2 with the reference constants (inertia := length, no armature or
    damping) through the chain kernel reproduces the reference's golden steps
    (control.py:67-152) — same tolerances as tests/test_gpu_parity.py;
  * n = 7 (build-defined model, parity unpinned by the reference) against the
    fp64 C chain oracle (oracle/chain_oracle.c, itself checked against the NumPy
    restatement and, at n = 2, the reference).

Tolerances at n = 7 (fp32 device vs fp64 oracle): the weighted noise / control
within 1e-4 of max(|.|, 1) (BASELINE.json); the same argmin; S at the 99th
percentile within 1e-5 at T <= 8 and 2e-4 at T = 32 and 128 (1e-7 when the exact
control-cost term dominates S, lambda = 1e9); at most 0.2 % of the samples
beyond 1e-3, and each of those explained by nearest-waypoint ties
(tests/tieflip.py): xydq_circle.txt starts with waypoints 6e-5 m apart whose dq
columns step by ~2e-3, and one fp32 step rounds the joint angles to ~2e-7 rad,
so where the fp64 end effector lies within a few um of the bisector of two
slots, the fp32 one may pick the neighbour (the same with OCML sincosf:
measured, tools/chain_cost_check.py); the device S then equals the fp64 S with
the neighbour's stage cost at that step.  At n = 7 this is checked exactly: the
kernel's slot-recording build (ChainEngine.debug_slots, same bits) reports the
slot it picked at every step, and the fp64 cost recomputed with those picks
must equal the device's S to 1e-4, with every pick that differs from the fp64
argmin a tie within PICK_GAP_M; the other link counts use the flip search.
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import chain_oracle as CO  # noqa: E402
import coracle  # noqa: E402
from conftest import STEP_FIXTURES, load_step, record  # noqa: E402
from tieflip import device_pick_residual, tie_flip_residual  # noqa: E402

U_TOL = 1e-4
S_TOL = 5e-5
TIE_GAP_M = 1e-5   # a tie: the two nearest slots' distances within 10 um of each other (the slots are 60 um apart)
PICK_GAP_M = 1e-6  # a pick the device makes differently from fp64: the two distances within 1 um (measured <= 0.34 um)
W, TW = [0.5, 0.5, 5.0, 5.0], [5.0, 5.0, 50.0, 50.0]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


def _urel(a, b):
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def _c5():
    from mppi_robotarm_amd.chain import CHAIN7_SIGMA, CHAIN7_X0, ChainParams, gravity_torque
    return ChainParams(), CHAIN7_X0, CHAIN7_SIGMA, gravity_torque(CHAIN7_X0[:7])


def _engine(K, T, lam=100.0, **kw):
    from mppi_robotarm_amd.chain import ChainEngine
    P, _, sig, _ = _c5()
    return ChainEngine(K, T, 0.006, lam, 0.98, sig, W, TW, kw.pop("expl", 0.0), kw.pop("chain", P), device=0, **kw)


@pytest.mark.parametrize("name", STEP_FIXTURES)
def test_chain_at_n2_reproduces_reference_steps(name, paths):
    from mppi_robotarm_amd.chain import ChainMPPIController, ChainParams
    g = load_step(name)
    c = ChainMPPIController(float(g["delta_t"]), paths[str(g["path"])], int(g["T"]), int(g["K"]),
                            float(g["param_exploration"]), float(g["param_lambda"]), float(g["param_alpha"]),
                            g["sigma"], g["stage_cost_weight"], g["terminal_cost_weight"],
                            visualze_sampled_trajs="sampled_traj" in g, chain=ChainParams.from_arm2(),
                            u_init=g["u_prev"])
    c.prev_waypoints_idx = int(g["prev_idx"])
    eps = g["eps"].astype(np.float64)
    c._calc_epsilon = lambda *a, **k: eps
    c.keep_costs = True
    u0, u_seq, opt, samp = c.calc_control_input(g["x0"])
    S = c.last_S
    assert int(np.argmin(S)) == int(np.argmin(g["S"]))
    assert float(np.max(np.abs(S - g["S"]) / np.abs(g["S"]))) < S_TOL
    assert _urel(u_seq, g["u_seq"]) < U_TOL
    assert c.prev_waypoints_idx == int(g["prev_idx_after"])
    np.testing.assert_allclose(opt, g["optimal_traj"], rtol=1e-4, atol=1e-4)   # dim_x = 4 at n = 2
    if "sampled_traj" in g:
        np.testing.assert_allclose(samp, g["sampled_traj"], rtol=1e-4, atol=1e-4)
    c.close()


@pytest.mark.parametrize("K,T,lam,s99,lps", [(4096, 32, 100.0, 2e-4, 1), (4096, 32, 100.0, 2e-4, 4),
                                            (4096, 32, 1.0e9, 1e-7, 1), (4096, 32, 1.0e9, 1e-7, 4),
                                            (131072, 128, 100.0, 2e-4, 1), (16384, 128, 100.0, 2e-4, 4),
                                            (32768, 128, 100.0, 2e-4, 4),   # the quad at auto's upper bound
                                            (3000, 7, 100.0, 1e-5, 1), (3000, 7, 100.0, 1e-5, 4)])
def test_chain_n7_against_c_oracle(K, T, lam, s99, lps, paths):
    """Config 5 (K=131072 T=128), its 8-way shard (K=16384, a quad per sample) and smaller shapes: S and the
    weighted noise vs fp64.

    Achieved on MI355X (profiles/r11/parity_records.jsonl): at config 5, S rel-err p50 1.9e-6, p99 1.0e-4,
    34 samples beyond 1e-3 (max 1.8e-3); recomputed in fp64 with the device's own window picks (the outliers
    plus 2048 random samples) every S agrees to 2.5e-5, and the 441 picks that differ from the fp64 argmin are
    all ties within 0.25 um (0.34 um for the quad-per-sample shard); w_eps exact (one-hot).  The fp32 states
    stay within 7e-6 rad of fp64 over the 128 steps (tools/c5_dense.py); the outliers are the cost's
    discontinuity at the ties."""
    P, x0, sig, ug = _c5()
    eng = _engine(K, T, lam, lanes_per_sample=lps)
    assert eng.lanes_per_sample == lps
    win = paths["xydq_circle"][:30]
    u = np.tile(ug, (T, 1)) + np.random.default_rng(4).normal(0, 0.3, (T, 7))
    eng.set_step_inputs(x0, win, u)
    noise = eng.philox_noise(11, 2)
    S_dev = torch.empty(K, dtype=torch.float64, device="cuda")
    eng.rollout(noise, S_out=S_dev)
    w = eng.weighted_noise()
    S = S_dev.cpu().numpy()
    nz = noise.cpu().numpy().transpose(0, 2, 1)   # device [T][K][n] -> (T, n, K)
    Sr = coracle.chain_rollout_costs(x0, u, nz, win, 0.006, lam, 0.98, sig, W, TW, CO.ChainParams(), layout="TNK")
    _, wr = coracle.chain_weighted_noise(Sr, nz, lam, layout="TNK")
    rel = np.abs(S - Sr) / np.abs(Sr)
    print(f"chain n=7 K={K} T={T} lam={lam:g} lps={lps}: S rel-err p50 {np.median(rel):.2e} p99 {np.percentile(rel, 99):.2e} "
          f"max {rel.max():.2e}, frac > 1e-3 {np.mean(rel > 1e-3):.2e}, w_eps rel-err {_urel(w, wr):.2e}")
    record("chain_n7", K=K, T=T, lam=lam, lps=lps, S_p50=float(np.median(rel)), S_p99=float(np.percentile(rel, 99)),
           S_max=float(rel.max()), frac_above_1e3=float(np.mean(rel > 1e-3)), w_eps_rel_err=_urel(w, wr))
    assert np.all(np.isfinite(S))
    assert int(np.argmin(S)) == int(np.argmin(Sr))
    assert float(np.percentile(rel, 99)) < s99
    assert float(np.mean(rel > 1e-3)) <= 2e-3   # the tie rate (measured 0 - 0.1 %), each tie checked below
    # every sample beyond 1e-3 is a nearest-waypoint tie: the same launch through the
    # slot-recording build gives the same bits and the slot it picked at every step;
    # the fp64 cost with those picks equals the device's, and every pick that differs
    # from the fp64 argmin is a tie (the two slots' distances within TIE_GAP_M)
    S2 = torch.empty(K, dtype=torch.float64, device="cuda")
    slots = eng.debug_slots(noise, S_out=S2)
    assert np.array_equal(S2.cpu().numpy(), S)
    assert slots.min() >= 0 and slots.max() < 30
    out = np.flatnonzero(rel > 1e-3)
    check = np.union1d(out, np.random.default_rng(5).choice(K, min(K, 2048), replace=False))
    res, gap, nd = device_pick_residual(S, Sr, check, x0, u, nz, win, 0.006, W, TW, CO.ChainParams(), slots)
    print(f"   {len(out)} samples beyond 1e-3; {len(check)} samples recomputed with the device's picks: residual max "
          f"{res.max():.2e}, {int(nd.sum())} picks differ from fp64 (in {int(np.count_nonzero(nd))} samples), "
          f"largest gap {gap.max():.2e} m")
    record("chain_n7_ties", K=K, T=T, lam=lam, lps=lps, n_beyond_1e3=int(len(out)), n_checked=int(len(check)),
           residual_max=float(res.max()), picks_differing=int(nd.sum()), gap_max_m=float(gap.max()))
    assert res.max() < min(s99, 1e-4) and gap.max() < PICK_GAP_M
    assert _urel(w, wr) < U_TOL
    eng.close()


def _fused(eng, paths, noises, u0):
    from mppi_robotarm_amd.chain import CHAIN7_X0
    eng.set_step_inputs(CHAIN7_X0, paths["xydq_circle"][2:32], u0)
    out = []
    for nz in noises:
        eng.rollout(nz, fused_update=True)
        out.append((eng.weighted_noise(), eng.nominal()))
    return out


@pytest.mark.parametrize("lam,lps", [(100.0, 1), (1.0e9, 1), (100.0, 4)])
def test_chain_handoff_forms_are_bit_identical(lam, lps, paths, monkeypatch):
    K, T = 32768 // lps, 48
    _, _, _, ug = _c5()
    runs = {}
    for form in ("poll", "counter"):
        if form == "counter":
            monkeypatch.setenv("MPPI_HANDOFF", "counter")
        eng = _engine(K, T, lam, lanes_per_sample=lps)
        assert eng.handoff == form
        noises = [eng.philox_noise(5, s) for s in range(3)]
        runs[form] = _fused(eng, paths, noises, np.tile(ug, (T, 1)))
        eng.close()
    for (wp, up), (wc, uc) in zip(runs["poll"], runs["counter"]):
        assert np.array_equal(wp, wc) and np.array_equal(up, uc)


@pytest.mark.parametrize("precision,lps", [("f32", 1), ("f32", 4), ("f64", 1)])
def test_chain_fused_update_matches_host_update(precision, lps, paths):
    from scipy.ndimage import median_filter
    K, T = 8192, 40
    _, _, _, ug = _c5()
    u = np.tile(ug, (T, 1)) + np.random.default_rng(1).normal(0, 0.5, (T, 7))
    eng = _engine(K, T, 1.0e6, precision=precision, lanes_per_sample=lps)
    noise = eng.philox_noise(9, 0)
    from mppi_robotarm_amd.chain import CHAIN7_X0
    eng.set_step_inputs(CHAIN7_X0, paths["xydq_circle"][:30], u)
    eng.rollout(noise)
    w = eng.weighted_noise()
    filt = np.stack([median_filter(w[:, d], size=10, mode="reflect") for d in range(7)], 1)
    un = u + filt
    expect = np.vstack([un[1:], un[-1:]])                       # control.py:148-149
    eng.set_step_inputs(CHAIN7_X0, paths["xydq_circle"][:30], u)
    eng.rollout(noise, fused_update=True)
    np.testing.assert_allclose(eng.nominal(), expect, rtol=1e-12, atol=1e-12)
    # the next launch on the device-written nominal (u and the control-cost rows a_t) equals one on the
    # host-uploaded nominal
    S1 = torch.empty(K, dtype=torch.float64, device="cuda")
    eng.rollout(noise, S_out=S1)
    S1 = S1.cpu().numpy()
    eng.set_step_inputs(CHAIN7_X0, paths["xydq_circle"][:30], eng.nominal())
    S2 = torch.empty(K, dtype=torch.float64, device="cuda")
    eng.rollout(noise, S_out=S2)
    np.testing.assert_allclose(S1, S2.cpu().numpy(), rtol=1e-12 if precision == "f64" else 1e-6)
    eng.close()


def test_chain_shards_and_device_merge(paths):
    """Virtual shards (Philox slices of the unsharded draw) + device merge == unsharded."""
    K, T, G = 12288, 24, 3
    _, x0, _, ug = _c5()
    u = np.tile(ug, (T, 1))
    full = _engine(K, T, 1.0e7)
    full.set_step_inputs(x0, paths["xydq_circle"][:30], u)
    noise = full.philox_noise(21, 4)
    full.rollout(noise)
    w_full = full.weighted_noise()
    Kl = K // G
    parts = torch.empty(G * full.partial_len, dtype=torch.float64, device="cuda")
    engs = []
    for g in range(G):
        e = _engine(Kl, T, 1.0e7, K_total=K, k_offset=g * Kl)
        e.set_step_inputs(x0, paths["xydq_circle"][:30], u)
        nz = e.philox_noise(21, 4)
        assert torch.equal(nz, noise[:, g * Kl:(g + 1) * Kl, :])
        e.rollout(nz, partial_out=parts[g * e.partial_len:(g + 1) * e.partial_len])
        engs.append(e)
    engs[0].merge(parts, G)
    np.testing.assert_allclose(engs[0].weighted_noise(), w_full, rtol=1e-10, atol=1e-12)
    for e in engs + [full]:
        e.close()


def test_chain_philox_noise_has_covariance_sigma():
    K, T = 65536, 4
    _, _, sig, _ = _c5()
    eng = _engine(K, T)
    z = eng.philox_noise(3, 0).cpu().numpy()                    # (T, K, 7)
    x = z.reshape(-1, 7).astype(np.float64)
    assert np.max(np.abs(x.mean(0))) < 0.05
    cov = np.cov(x.T)
    np.testing.assert_allclose(cov, sig, atol=0.1 * np.sqrt(np.outer(np.diag(sig), np.diag(sig))).max() / 4)
    eng.close()


def test_chain_trajectories_match_oracle(paths):
    K, T = 64, 20
    P, x0, _, ug = _c5()
    eng = _engine(K, T)
    u = np.tile(ug, (T, 1))
    eng.set_step_inputs(x0, paths["xydq_circle"][:30], u)
    noise = eng.philox_noise(2, 0)
    tr = eng.trajectories(base_u=u, noise=noise).double().cpu().numpy()
    nz = noise.cpu().numpy().transpose(0, 2, 1)   # device [T][K][n] -> (T, n, K)
    ctrl = np.roll(u[None] + nz.transpose(2, 0, 1), 1, axis=1)    # control(t) = u[t-1] + eps[t-1]
    ref = coracle.chain_traj(x0, ctrl, 0.006, CO.ChainParams())
    np.testing.assert_allclose(tr, ref, rtol=1e-4, atol=1e-4)
    eng.close()


def test_chain_errors():
    from mppi_robotarm_amd.chain import CHAIN7_SIGMA, ChainEngine, ChainParams
    with pytest.raises(np.linalg.LinAlgError):
        ChainEngine(256, 8, 0.006, 100.0, 0.98, -np.eye(7), W, TW, device=0)
    with pytest.raises(ValueError):
        ChainEngine(256, 8, 0.006, 100.0, 0.98, np.eye(8), W, TW, chain=ChainParams(*(tuple([1.0] * 8),) * 7),
                    device=0)
    # a quad per sample addresses its noise with 32-bit buffer offsets: K T n 4 bytes must stay below 2^31
    big = 600000   # 600000 * 128 * 7 * 4 B = 2.15 GB
    with pytest.raises(ValueError, match="lanes_per_sample 4"):
        ChainEngine(big, 128, 0.006, 100.0, 0.98, CHAIN7_SIGMA, W, TW, device=0, lanes_per_sample=4)
    e = ChainEngine(32768, 128, 0.006, 100.0, 0.98, CHAIN7_SIGMA, W, TW, device=0, lanes_per_sample=4)
    assert e.lanes_per_sample == 4   # 117 MB of noise: allowed
    e.close()


def _uniform_chain(mod, n):
    """n uniform slender links of 1 kg and 2 m total reach (config 5's arm at n = 7)."""
    L = 2.0 / n
    return mod.ChainParams(m=(1.0,) * n, l=(L,) * n, lc=(L / 2,) * n, I=(L * L / 12.0,) * n, fk=(L,) * n,
                           J=(0.1,) * n, b=(1.0,) * n)


def _link_case(n, K, T, lam, paths, precision="f32", lps=1):
    """A uniform n-link chain with a random SPD Sigma, gravity-holding nominal plus noise and a window away from
    the path start, through the engine and the C fp64 chain oracle: (S, S_ref, w_eps, w_eps_ref, tie inputs)."""
    from mppi_robotarm_amd.chain import ChainEngine, ChainParams, gravity_torque
    rng = np.random.default_rng(n * 100 + T)
    import mppi_robotarm_amd.chain as chain_mod
    P, Po = _uniform_chain(chain_mod, n), _uniform_chain(CO, n)
    assert isinstance(P, ChainParams)
    q = np.array([1.4] + [-2.2 / (n - 1)] * (n - 1)) if n > 1 else np.array([1.4])
    x0 = np.concatenate([q, rng.normal(0, 0.2, n)])
    A = rng.normal(0, 1, (n, n))
    sig = A @ A.T / n + np.diag(np.linspace(8.0, 1.0, n))
    u = np.tile(gravity_torque(q, P), (T, 1)) + rng.normal(0, 0.3, (T, n))
    eng = ChainEngine(K, T, 0.006, lam, 0.98, sig, W, TW, 0.0, P, device=0, precision=precision,
                      lanes_per_sample=lps)
    win = paths["xydq_circle"][40:70]
    eng.set_step_inputs(x0, win, u)
    noise = eng.philox_noise(3 + n, 1)
    S_dev = torch.empty(K, dtype=torch.float64, device="cuda")
    eng.rollout(noise, S_out=S_dev)
    w = eng.weighted_noise()
    S = S_dev.cpu().numpy()
    nz = noise.cpu().numpy().transpose(0, 2, 1)   # device [T][K][n] -> (T, n, K)
    eng.close()
    Sr = coracle.chain_rollout_costs(x0, u, nz, win, 0.006, lam, 0.98, sig, W, TW, Po, layout="TNK")
    _, wr = coracle.chain_weighted_noise(Sr, nz, lam, layout="TNK")
    return S, Sr, w, wr, (x0, u, nz, win, Po)


LINK_CASES = [(3, 256, 16, 100.0), (4, 3000, 24, 100.0), (5, 777, 32, 1.0e4), (6, 2048, 20, 100.0),
              (7, 1000, 9, 1.0e8), (2, 513, 40, 100.0)]


@pytest.mark.parametrize("lps", [1, 4])
@pytest.mark.parametrize("n,K,T,lam", LINK_CASES)
def test_chain_every_link_count_against_c_oracle(n, K, T, lam, lps, paths):
    """Every compiled chain length (chain_rollout_kernel<N>, N = 2..7), one lane per sample and a quad per
    sample, against the C fp64 chain oracle."""
    S, Sr, w, wr, tie = _link_case(n, K, T, lam, paths, lps=lps)
    rel = np.abs(S - Sr) / np.abs(Sr)
    print(f"chain n={n} K={K} T={T} lps={lps}: S rel-err p99 {np.percentile(rel, 99):.2e} max {rel.max():.2e}, "
          f"w_eps {_urel(w, wr):.2e}")
    assert np.all(np.isfinite(S))
    j, jr = int(np.argmin(S)), int(np.argmin(Sr))
    assert j == jr or abs(Sr[j] - Sr[jr]) <= 1e-5 * abs(Sr[jr])
    assert float(np.percentile(rel, 99)) < 2e-4
    out = np.flatnonzero(rel > 1e-3)   # nearest-waypoint ties only (tests/tieflip.py)
    if len(out):
        x0, u, nz, win, Po = tie
        res, gap = tie_flip_residual(S, Sr, out, x0, u, nz, win, 0.006, W, TW, Po)
        assert res.max() < 2e-4 and gap.max() < TIE_GAP_M
    assert _urel(w, wr) < U_TOL


@pytest.mark.parametrize("n,K,T,lam", LINK_CASES)
def test_chain_f64_every_link_count_against_c_oracle(n, K, T, lam, paths):
    """The fp64 rollout (precision="f64", ChainStateD) against the same oracle: equal to rounding."""
    S, Sr, w, wr, _ = _link_case(n, K, T, lam, paths, precision="f64", lps=1)
    rel = np.abs(S - Sr) / np.abs(Sr)
    print(f"chain f64 n={n} K={K} T={T}: S rel-err max {rel.max():.2e}, w_eps {_urel(w, wr):.2e}")
    record("chain_f64", n=n, K=K, T=T, lam=lam, S_max=float(rel.max()), w_eps_rel_err=_urel(w, wr))
    assert int(np.argmin(S)) == int(np.argmin(Sr))
    assert float(rel.max()) < 1e-11
    assert _urel(w, wr) < 1e-10


def test_chain_c5_spread_weights(paths):
    """Config 5's size (K=131072, T=128) with lambda = 3e5, where the fp64 weights spread over ESS >= 10
    samples: the fp64 rollout holds w_eps to 1e-4 of the C oracle (BASELINE.json); the fp32 rollout's error is
    recorded beside it (its nearest-waypoint ties among the weighted samples move w_eps)."""
    K, T, lam = 131072, 128, 3.0e5
    _, x0, sig, ug = _c5()
    win = paths["xydq_circle"][:30]
    u = np.tile(ug, (T, 1))
    errs = {}
    for prec in ("f64", "f32"):
        eng = _engine(K, T, lam, precision=prec, lanes_per_sample=1)
        eng.set_step_inputs(x0, win, u)
        noise = eng.philox_noise(11, 2)
        S_dev = torch.empty(K, dtype=torch.float64, device="cuda")
        eng.rollout(noise, S_out=S_dev)
        w = eng.weighted_noise()
        S = S_dev.cpu().numpy()
        nz = noise.cpu().numpy().transpose(0, 2, 1)   # device [T][K][n] -> (T, n, K)
        eng.close()
        if prec == "f64":
            Sr = coracle.chain_rollout_costs(x0, u, nz, win, 0.006, lam, 0.98, sig, W, TW, CO.ChainParams(),
                                             layout="TNK")
            _, wr = coracle.chain_weighted_noise(Sr, nz, lam, layout="TNK")
            wt = np.exp(-(Sr - Sr.min()) / lam)
            ess = float(wt.sum() ** 2 / (wt ** 2).sum())
        errs[prec] = (_urel(w, wr), float(np.max(np.abs(S - Sr) / np.abs(Sr))))
    print(f"c5 lambda={lam:g}: ESS {ess:.1f}; w_eps rel-err f64 {errs['f64'][0]:.2e} (S max {errs['f64'][1]:.2e}), "
          f"f32 {errs['f32'][0]:.2e} (S max {errs['f32'][1]:.2e})")
    record("chain_c5_spread", K=K, T=T, lam=lam, ess=ess, w_eps_rel_err_f64=errs["f64"][0],
           S_max_f64=errs["f64"][1], w_eps_rel_err_f32=errs["f32"][0], S_max_f32=errs["f32"][1])
    assert ess >= 10.0
    assert errs["f64"][0] < U_TOL and errs["f64"][1] < 1e-11

    # the default controller (precision="auto") on the same step: its fp32 rollout sees eta - 1 > ETA_TOL and
    # the step is run again in fp64, so the update holds 1e-4 against the oracle's; the next step, still
    # spread, goes straight to fp64.  Wall time per call recorded beside fp32 alone (the switch's cost).
    import time

    from scipy.ndimage import median_filter
    from mppi_robotarm_amd.chain import ChainMPPIController
    wm = np.stack([median_filter(wr[:, d], size=10, mode="reflect") for d in range(7)], axis=1)
    un = u + wm
    u_ref = np.concatenate([un[1:], un[-1:]])          # control.py:126, 148-149
    kw = dict(device=0, verbose=False, noise="device", seed=11, u_init=u.copy())
    ctl = {p: ChainMPPIController(0.006, paths["xydq_circle"], T, K, 0.0, lam, 0.98, sig, precision=p, **kw)
           for p in ("auto", "f32")}
    res, wall = {}, {}
    for p, c in ctl.items():
        c._step_count = 2                                  # the stream position of the draw above (seed 11, step 2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, u_seq, _, _ = c.calc_control_input(x0.copy())
        wall[p] = [time.perf_counter() - t0]
        res[p] = (_urel(u_seq, u_ref), c.last_precision, c.last_eta)
        for _ in range(3):                                 # the following steps, back to back
            t0 = time.perf_counter()
            c.calc_control_input(x0.copy())
            wall[p].append(time.perf_counter() - t0)
        c.close()
    print(f"auto controller: u rel-err {res['auto'][0]:.2e} ({res['auto'][1]}, eta {res['auto'][2]:.3f}), "
          f"f32 controller {res['f32'][0]:.2e}; wall ms auto {[round(w * 1e3, 2) for w in wall['auto']]} "
          f"f32 {[round(w * 1e3, 2) for w in wall['f32']]}")
    record("chain_c5_spread_auto", u_rel_err_auto=res["auto"][0], u_rel_err_f32=res["f32"][0], eta=res["auto"][2],
           wall_ms_auto=[w * 1e3 for w in wall["auto"]], wall_ms_f32=[w * 1e3 for w in wall["f32"]])
    assert res["auto"][1] == "f64" and res["auto"][2] - 1.0 > ChainMPPIController.ETA_TOL
    assert res["auto"][0] < U_TOL


def test_chain_lanes_per_sample_agree(paths):
    """A quad per sample and one lane per sample on the same inputs: S within the fp32 bound each keeps against
    the fp64 oracle (p99 2e-4, test_chain_n7_against_c_oracle: the quad steps in absolute angles and sums the
    control-cost terms in another order, so its roundings, and the nearest-waypoint ties they tip, are its own),
    the same argmin, w_eps within 1e-4; auto picks 4 at the 8-way shard of config 5 (K = 16384) and 1 at the
    full K."""
    K, T, lam = 16384, 64, 100.0
    _, x0, _, ug = _c5()
    win = paths["xydq_circle"][:30]
    u = np.tile(ug, (T, 1)) + np.random.default_rng(8).normal(0, 0.3, (T, 7))
    out = {}
    for lps in (1, 4):
        eng = _engine(K, T, lam, lanes_per_sample=lps)
        eng.set_step_inputs(x0, win, u)
        noise = eng.philox_noise(12, 0)
        S_dev = torch.empty(K, dtype=torch.float64, device="cuda")
        eng.rollout(noise, S_out=S_dev)
        out[lps] = (S_dev.cpu().numpy(), eng.weighted_noise())
        eng.close()
    rel = np.abs(out[4][0] - out[1][0]) / np.abs(out[1][0])
    print(f"lps 4 vs 1: S rel p99 {np.percentile(rel, 99):.2e} max {rel.max():.2e}, "
          f"w_eps {_urel(out[4][1], out[1][1]):.2e}")
    assert int(np.argmin(out[4][0])) == int(np.argmin(out[1][0]))
    assert float(np.percentile(rel, 99)) < 2e-4
    assert _urel(out[4][1], out[1][1]) < U_TOL
    assert _engine(16384, 8).lanes_per_sample == 4 and _engine(131072, 8).lanes_per_sample == 1


@pytest.mark.parametrize("T", [1, 2, 3, 5, 6])
@pytest.mark.parametrize("precision,lps", [("f32", 1), ("f32", 4), ("f64", 1)])
def test_chain_short_horizons(T, precision, lps, paths):
    """Horizons shorter than the prefetch rings and the 2- / 4-step unrolls (the remainder steps alone; with a
    quad per sample, step 0 is peeled and T = 5 is exactly one 4-step iteration, T = 6 one plus a remainder),
    ragged K, against the C fp64 chain oracle."""
    K, lam = 999, 100.0
    _, x0, sig, ug = _c5()
    win = paths["xydq_circle"][:30]
    u = np.tile(ug, (T, 1)) + np.random.default_rng(T).normal(0, 0.3, (T, 7))
    eng = _engine(K, T, lam, precision=precision, lanes_per_sample=lps)
    eng.set_step_inputs(x0, win, u)
    noise = eng.philox_noise(21, T)
    S_dev = torch.empty(K, dtype=torch.float64, device="cuda")
    eng.rollout(noise, S_out=S_dev)
    w = eng.weighted_noise()
    S = S_dev.cpu().numpy()
    nz = noise.cpu().numpy().transpose(0, 2, 1)   # device [T][K][n] -> (T, n, K)
    eng.close()
    Sr = coracle.chain_rollout_costs(x0, u, nz, win, 0.006, lam, 0.98, sig, W, TW, CO.ChainParams(), layout="TNK")
    _, wr = coracle.chain_weighted_noise(Sr, nz, lam, layout="TNK")
    rel = np.abs(S - Sr) / np.abs(Sr)
    bound = 1e-11 if precision == "f64" else 1e-5
    assert int(np.argmin(S)) == int(np.argmin(Sr))
    assert float(np.percentile(rel, 99)) < bound
    assert _urel(w, wr) < (1e-10 if precision == "f64" else U_TOL)


def test_chain_controller_rereads_its_parameters(paths):
    """ChainMPPIController follows what a call reads, as the 2-DoF drop-in does: K, T, Sigma (in place or
    rebound), lambda (gamma kept from construction, control.py:45), the cost weights, the exploration split
    and delta_t changed between calls act on the next step exactly as a controller built with them would."""
    from mppi_robotarm_amd.chain import CHAIN7_X0, ChainMPPIController, gravity_torque
    _, x0, sig, ug = _c5()
    kw = dict(device=0, verbose=False, noise="numpy")
    c = ChainMPPIController(0.006, paths["xydq_circle"], 16, 2048, 0.0, 100.0, 0.98, sig.copy(), u_init=ug, **kw)
    np.random.seed(1)
    c.calc_control_input(x0)
    edits = [
        lambda o: o.Sigma.__setitem__((0, 0), o.Sigma[0, 0] * 1.5),
        lambda o: setattr(o, "param_lambda", 40.0),
        lambda o: setattr(o, "stage_cost_weight", np.array([0.5, 1.0, 5.0, 5.0])),
        lambda o: setattr(o, "param_exploration", 0.25),
        lambda o: (setattr(o, "K", 1000), setattr(o, "T", 12), setattr(o, "u_prev", np.tile(ug, (12, 1)))),
        lambda o: setattr(o, "delta_t", 0.005),
    ]
    for i, edit in enumerate(edits):
        edit(c)
        ref = ChainMPPIController(c.delta_t, paths["xydq_circle"], c.T, c.K, c.param_exploration, 100.0, 0.98,
                                  c.Sigma.copy(), c.stage_cost_weight, c.terminal_cost_weight, u_init=c.u_prev.copy(), **kw)
        ref.param_lambda = c.param_lambda                   # gamma from lambda = 100, as c's
        ref.prev_waypoints_idx = c.prev_waypoints_idx
        np.random.seed(10 + i)
        got = c.calc_control_input(x0)
        np.random.seed(10 + i)
        want = ref.calc_control_input(x0)
        assert np.array_equal(got[1], want[1]), i
        ref.close()
    c.close()


def test_chain_fused_dropin_equals_host_update_path(paths):
    """ChainMPPIController's one-launch step (update on the device, one read-back, fp64 optimal trajectory on
    the host, next noise prefetched) against the host-update path (w_eps read back, SciPy median, u += w_eps)
    from the same state and noise: u, the aliasing and the optimal trajectory bit for bit over a few ticks, one
    of them after an in-place edit of u_prev (the fused path skips re-staging only an unchanged nominal)."""
    from mppi_robotarm_amd.chain import ChainMPPIController
    _, x0, sig, ug = _c5()
    kw = dict(device=0, verbose=False, noise="device", seed=4)
    # the oracle side of the trajectory is test_chain_optimal_traj_host_against_oracle
    fused = ChainMPPIController(0.006, paths["xydq_circle"], 24, 4096, 0.0, 100.0, 0.98, sig, u_init=ug, **kw)
    host = ChainMPPIController(0.006, paths["xydq_circle"], 24, 4096, 0.0, 100.0, 0.98, sig, u_init=ug,
                               visualze_sampled_trajs=True, **kw)   # takes the host-update path
    x = x0.copy()
    for tick in range(5):
        if tick == 2:
            for c in (fused, host):
                c.u_prev += 0.1                  # an in-place edit of the nominal must be staged, not skipped
        outs = []
        for c in (fused, host):
            u_prev = c.u_prev
            u0, u_seq, opt, samp = c.calc_control_input(x)
            assert u_seq is u_prev and np.shares_memory(u0, u_prev)
            outs.append((u_seq.copy(), opt.copy(), c.prev_waypoints_idx))
        (ua, oa, ia), (ub, ob, ib) = outs
        assert ia == ib and np.array_equal(ua, ub), tick
        assert np.array_equal(oa, ob), tick
        x = oa[3].copy()
    fused.close()
    host.close()


def test_chain_optimal_traj_host_against_oracle():
    """mppi_chain_optimal_traj_host (fp64 ChainStateD on the host) against the fp64 chain oracle's dynamics:
    x_{t+1} = F(x_t, u_new[t - 1]), u_new[-1] at t = 0 (control.py:129-134), to 1e-12."""
    P, x0, sig, ug = _c5()
    T = 20
    eng = _engine(256, T)
    u_new = np.tile(ug, (T, 1)) + np.random.default_rng(9).normal(0, 0.5, (T, 7))
    got = eng.optimal_traj_host(x0, u_new)
    q, dq = x0[None, :7].copy(), x0[None, 7:].copy()
    want = np.zeros((T, 14))
    for t in range(T):
        q, dq = CO.chain_forward_dynamics(q, dq, u_new[t - 1][None, :], 0.006, CO.ChainParams())
        want[t, :7], want[t, 7:] = q[0], dq[0]
    # the hardware-fma instance and the baseline x86-64 one give the same bits (fma is exact in both,
    # nothing else is contracted on the host)
    os.environ["MPPI_HOST_FMA"] = "0"
    try:
        base = eng.optimal_traj_host(x0, u_new)
    finally:
        del os.environ["MPPI_HOST_FMA"]
    eng.close()
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12)
    assert np.array_equal(got.view(np.uint64), base.view(np.uint64))


def test_chain_debug_and_output_entry_points_refuse_misuse(paths):
    """The new chain entry points fail loudly with the reference's exception classes (MPPI_E_ARG ->
    ValueError): the fused outputs without a fused launch, after the nominal was re-staged, and the
    slot-recording build on a chain it is not built for (only 7 links)."""
    P, x0, sig, ug = _c5()
    eng = _engine(512, 8)
    win = paths["xydq_circle"][:30]
    u = np.tile(ug, (8, 1))
    eng.set_step_inputs(x0, win, u)
    noise = eng.philox_noise(1, 0)
    eng.rollout(noise)                                   # no fused update
    with pytest.raises(ValueError, match="fused"):
        eng.wait_outputs()
    eng.rollout(noise, fused_update=True, host_out=True)
    got, _ = eng.wait_outputs()
    assert got.shape == (8, 7) and np.all(np.isfinite(got))
    eng.set_step_inputs(x0, win, u + 1.0)                # a different nominal staged: no update to read
    with pytest.raises(ValueError, match="fused"):
        eng.wait_outputs()
    eng.close()
    from mppi_robotarm_amd.chain import ChainEngine, ChainParams
    e2 = ChainEngine(256, 8, 0.006, 100.0, 0.98, np.eye(2) * 20.0, W, TW, 0.0, ChainParams.from_arm2(), device=0)
    with pytest.raises(ValueError, match="7-link"):
        e2.debug_slots(e2.philox_noise(1, 0))
    e2.close()
