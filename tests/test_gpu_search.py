"""The window search through the candidate table (mppi_device.h TabSearch,
built per window by search_table_kernel) against the full 30-slot scan of the
same fp32 keys: the nearest slot of control.py:200-232 as the device computes
it must be bit-identical (argmin index) for every point, and whole rollouts
must give bit-identical S and w_eps with the table on (MPPI_SEARCH=table,
opt-in) and off (the default full scan).  Point sets aim at the table's weak spots: cell edges (the
diamond-angle and sigma bin boundaries), perpendicular bisectors of adjacent
waypoints (ties), the near field and the window itself, far points, truncated
windows at the path end, duplicated and scattered waypoints."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from test_gpu_parity import RUNPY, X0, _engine  # noqa: E402

PATHS = np.load(os.path.join(os.path.dirname(__file__), "golden", "paths.npz"))
KTAB_PHI, KTAB_SIG = 256, 32


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


def _windows():
    circ = PATHS["xydq_circle"][:, :4]
    traj = PATHS["trajectory"][:, :4]
    traj1 = PATHS["trajectory1"][:, :4]
    rng = np.random.default_rng(7)
    dup = np.repeat(circ[100:115], 2, axis=0)
    scat = np.concatenate([rng.uniform(-1.5, 1.5, (30, 2)), rng.normal(size=(30, 2))], axis=1)
    return {
        "circle0": circ[0:30], "circle500": circ[500:530], "circle_end": circ[1985:2000],
        "traj0": traj[0:30], "traj1500": traj[1500:1530], "traj1_700": traj1[700:730],
        "dup": dup, "scattered": scat, "w1": circ[10:11], "w2": circ[10:12],
    }


def _points(win, rng):
    xy = win[:, :2].astype(np.float32).astype(np.float64)
    c = xy.mean(0)
    R = max(float(np.max(np.linalg.norm(xy - c, axis=1))), 1e-6)
    pts = [rng.uniform(-2.0, 2.0, (20000, 2))]                      # the reach disk and beyond
    for s in (0.3, 1.0, 3.0, 10.0, 100.0):                         # near field .. far field
        pts.append(c + rng.normal(size=(4000, 2)) * R * s)
    pts.append(xy)                                                 # on the waypoints
    pts.append(c[None])
    if len(xy) > 1:                                                # bisectors of neighbours (ties)
        mid = 0.5 * (xy[1:] + xy[:-1])
        d = xy[1:] - xy[:-1]
        nrm = np.stack([-d[:, 1], d[:, 0]], 1)
        nrm /= np.maximum(np.linalg.norm(nrm, axis=1, keepdims=True), 1e-30)
        for dist in (0.0, R * 0.1, R, R * 10, 0.1, 1.0):
            for sgn in (1, -1):
                pts.append(mid + sgn * dist * nrm)
    # cell edges: diamond angle a = k * 4 / KTAB_PHI, sigma = sb / sscale, +- a few ulps
    sscale = KTAB_SIG * 0.5 * np.sqrt(np.max(np.sum((xy - c) ** 2, 1)))
    a = np.repeat(np.arange(KTAB_PHI + 1) * (4.0 / KTAB_PHI), 8)
    sb = rng.integers(1, KTAB_SIG + 1, a.shape)
    rho = max(sscale, 1e-6) / sb * (1 + rng.choice([-1e-6, 0, 1e-6], a.shape))
    a = np.mod(a + rng.choice([-1e-6, -1e-7, 0, 1e-7, 1e-6], a.shape), 4.0)
    q = np.floor(a)
    f = a - q
    dx = np.select([q == 0, q == 1, q == 2], [1 - f, -f, f - 1], f)
    dy = np.select([q == 0, q == 1, q == 2], [f, 1 - f, -f], f - 1)
    n = np.hypot(dx, dy)
    pts.append(np.stack([c[0] + rho * dx / n, c[1] + rho * dy / n], 1))
    return np.concatenate(pts, 0)


@pytest.mark.parametrize("name", list(_windows()))
def test_table_search_matches_full_scan(name):
    win = _windows()[name]
    eng = _with_search("table", lambda: _engine(65536, 16))
    try:
        assert eng.lanes_per_sample == 1
        eng.set_step_inputs(X0, win, np.tile([10.0, -2.0], (16, 1)))
        pts = _points(win, np.random.default_rng(abs(hash(name)) % 2 ** 32))
        out = eng.search_check(pts)
        bad = np.nonzero(out[:, 0] != out[:, 1])[0]
        assert bad.size == 0, f"{bad.size} mismatches, first at {pts[bad[0]]}: table {out[bad[0]]}"
        assert out[:, 1].min() >= 0 and out[:, 1].max() < len(win)
    finally:
        eng.close()


def _with_search(mode, make):
    old = os.environ.get("MPPI_SEARCH")
    if mode is None:
        os.environ.pop("MPPI_SEARCH", None)
    else:
        os.environ["MPPI_SEARCH"] = mode
    try:
        return make()
    finally:
        if old is None:
            os.environ.pop("MPPI_SEARCH", None)
        else:
            os.environ["MPPI_SEARCH"] = old


def _rollout(K, T, win, u, x0, table, seed=3):
    eng = _with_search("table" if table else None, lambda: _engine(K, T))
    try:
        eng.set_step_inputs(x0, win, u)
        noise = eng.philox_noise(seed)
        S = torch.empty(K, dtype=torch.float64, device=eng.device)
        eng.rollout(noise, S_out=S)
        w = eng.weighted_noise()
        return S.cpu().numpy(), w
    finally:
        eng.close()


@pytest.mark.parametrize("case", ["c3", "mid_path", "end_path", "T61"])
def test_rollout_bit_identical_with_and_without_table(case):
    circ = PATHS["xydq_circle"][:, :4]
    K, T, win, x0 = 65536, 64, circ[0:30], X0
    u = np.tile([10.0, -2.0], (T, 1))
    if case == "mid_path":
        win = circ[700:730]
        x0 = np.array([0.3, 1.1, 0.5, -0.4])
        u = np.tile([3.0, 1.0], (T, 1))
    elif case == "end_path":
        win = circ[1988:2000]
    elif case == "T61":
        T = 61
        u = np.tile([10.0, -2.0], (T, 1))
    S_tab, w_tab = _rollout(K, T, win, u, x0, table=True)
    S_full, w_full = _rollout(K, T, win, u, x0, table=False)
    assert np.array_equal(S_tab, S_full)
    assert np.array_equal(w_tab, w_full)


def test_table_is_opt_in():
    eng = _with_search(None, lambda: _engine(65536, 16))
    try:
        eng.set_step_inputs(X0, PATHS["xydq_circle"][:30, :4], np.tile([10.0, -2.0], (16, 1)))
        with pytest.raises(ValueError, match="candidate table"):
            eng.search_check(np.zeros((4, 2)))
    finally:
        eng.close()
