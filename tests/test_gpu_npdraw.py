"""GPU: the reference's noise stream drawn on the device (include/mppi_rocm.h mppi_np_*, engine.NpDeviceStream).

control.py:163 draws eps = np.random.multivariate_normal(mu, Sigma, (K, T)) on NumPy's legacy global RandomState.
The device draw must give NumPy's values bit for bit (after the fp32 rounding of the upload) in the engine's noise
layout, and leave the RNG state NumPy's draw leaves (key array, position, cached Gaussian).  The expected values
here are NumPy's own multivariate_normal from the same state (the reference's call, not a restatement).
Covered: config 3's size (8.4 M normals: ~4 % of the logs take glibc's near-1 branch), config 5's (117 M), config 2's, odd sample
counts, a state with a cached Gaussian and an odd count (the draw starts with it and leaves a new one), states at
arbitrary word positions, a Sigma whose transform permutes the components, rank slices, and the drop-in
controller with the device draw against the host draw over a closed loop.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nd():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    from mppi_robotarm_amd.engine import NpDeviceStream
    d = NpDeviceStream(torch.device("cuda", 0))
    yield d
    d.close()


def _numpy_draw(K, T, sigma):
    x = np.random.multivariate_normal(np.zeros(sigma.shape[0]), sigma, (K, T))
    return x.astype(np.float32), np.random.get_state()


def _device_draw(nd, K, T, sigma, k_offset=0, K_local=None):
    from mppi_robotarm_amd import hostrng
    du = sigma.shape[0]
    K_local = K if K_local is None else K_local
    plan = hostrng.device_plan(np.zeros(du), sigma)
    assert plan is not None, "np.dot's rounding of this transform is not the pinned model on this host"
    out = torch.full((T, K_local, du), float("nan"), dtype=torch.float32, device="cuda")
    nd.draw(np.random.get_state(), (K, T, du), plan, out, torch.cuda.current_stream().cuda_stream, k_offset, K_local,
            (K_local * du, du, 1))
    st = nd.result()
    return out.cpu().numpy(), st


def _same_state(a, b):
    return a[0] == b[0] and np.array_equal(a[1], b[1]) and a[2:] == b[2:]


CASES = [
    (65536, 64, 0, "runpy"),       # config 3
    (4096, 32, 1, "runpy"),        # config 2
    (4097, 33, 2, "runpy"),        # odd K and T
    (512, 64, 3, "permuted"),      # Sigma's transform swaps the components
    (128, 129, 4, "scaled"),       # just over the size the controller hands to the device
    (4097, 33, 6, "general"),      # a full 2 x 2 transform through np.dot's pinned rounding (hostrng.dot2_model)
    (65536, 64, 7, "general"),     # the same at config 3's size
    (3001, 17, 8, "general2"),
]
SIGMAS = {"runpy": np.eye(2) * 20.0, "permuted": np.diag([2.0, 9.0]), "scaled": np.diag([0.3, 7.0]),
          "general": np.array([[20.0, 6.0], [6.0, 12.0]]),    # the sigma_k128_t20 fixture's Sigma
          "general2": np.array([[2.0, -1.5], [-1.5, 3.0]])}


@pytest.mark.parametrize("K,T,seed,sig", CASES)
@pytest.mark.parametrize("start", ["fresh", "offset", "cached"])
def test_device_draw_equals_numpy(nd, K, T, seed, sig, start):
    sigma = SIGMAS[sig]
    np.random.seed(seed)
    if start == "offset":
        np.random.random_sample(seed * 37 + 101)          # the state mid key array
    elif start == "cached":
        np.random.standard_normal(3)                      # an odd count: a cached Gaussian
    st0 = np.random.get_state()
    want, st_want = _numpy_draw(K, T, sigma)
    np.random.set_state(st0)
    got, st_got = _device_draw(nd, K, T, sigma)
    assert st_got is not None
    np.testing.assert_array_equal(got, want.transpose(1, 0, 2))
    assert _same_state(st_got, st_want)


def test_device_draw_equals_numpy_config5(nd):
    """Config 5's draw (K = 131072, T = 128, the 7-link chain's diagonal Sigma: 117 M normals): the plan's P = 1024,
    491 generator streams (more twist workgroups than CUs), 38 k write workgroups; from a state mid key array."""
    from mppi_robotarm_amd.chain import CHAIN7_SIGMA
    K, T = 131072, 128
    np.random.seed(10)
    np.random.random_sample(333)
    st0 = np.random.get_state()
    want, st_want = _numpy_draw(K, T, CHAIN7_SIGMA)
    want = np.ascontiguousarray(want.transpose(1, 0, 2))
    np.random.set_state(st0)
    got, st_got = _device_draw(nd, K, T, CHAIN7_SIGMA)
    assert st_got is not None
    np.testing.assert_array_equal(got, want)
    assert _same_state(st_got, st_want)


@pytest.mark.parametrize("sizes", [((65536, 64), (4096, 32)), ((4096, 32), (65536, 64)), ((65536, 64), (65536, 64))])
def test_consecutive_draws_continue_numpy(nd, sizes):
    """A draw that starts where the last one ended reads its jump sequence from the last draw's words (no fresh
    twist) unless the word buffer had to grow (small then large): every case equals NumPy's consecutive draws."""
    sigma = SIGMAS["runpy"]
    np.random.seed(12)
    st0 = np.random.get_state()
    wants = [_numpy_draw(K, T, sigma) for K, T in sizes]
    np.random.set_state(st0)
    for (K, T), (want, st_want) in zip(sizes, wants):
        got, st_got = _device_draw(nd, K, T, sigma)
        assert st_got is not None
        np.testing.assert_array_equal(got, want.transpose(1, 0, 2))
        assert _same_state(st_got, st_want)
        np.random.set_state(st_got)


def test_odd_normal_count_leaves_the_cached_gaussian(nd):
    """du = 1 and an odd K T: the draw ends on half a pair; NumPy caches f x1 for the next call."""
    sigma = np.array([[4.0]])
    np.random.seed(9)
    st0 = np.random.get_state()
    want, st_want = _numpy_draw(257, 129, sigma)
    assert st_want[3] == 1
    np.random.set_state(st0)
    got, st_got = _device_draw(nd, 257, 129, sigma)
    np.testing.assert_array_equal(got, want.transpose(1, 0, 2))
    assert _same_state(st_got, st_want)


def test_rank_slices_are_slices_of_the_whole_draw(nd):
    K, T, sigma = 3000, 20, SIGMAS["runpy"]
    np.random.seed(5)
    st0 = np.random.get_state()
    full, st_full = _device_draw(nd, K, T, sigma)
    for off, kl in ((0, 1000), (1000, 1001), (2001, 999)):
        np.random.set_state(st0)
        part, st_part = _device_draw(nd, K, T, sigma, off, kl)
        np.testing.assert_array_equal(part, full[:, off:off + kl])
        assert _same_state(st_part, st_full)   # every rank leaves the same state


def _loop(device_draw: bool, ticks=4, K=4096, T=32, between=None, sigma=None):
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    from mppi_robotarm_amd.params import X0_RUNPY, runpy_config
    from conftest import load_paths
    kw = runpy_config()
    kw.update(number_of_samples_K=K, horizon_step_T=T, visualze_sampled_trajs=False)
    if sigma is not None:
        kw["sigma"] = sigma
    c = MPPIControllerForPathTracking(ref_path=load_paths()["xydq_circle"], verbose=False, device=0,
                                      numpy_noise_on_device=device_draw, **kw)
    np.random.seed(21)
    x, out = X0_RUNPY.copy(), []
    for i in range(ticks):
        if between is not None:
            between(i, c)
        u0, u_seq, opt, _ = c.calc_control_input(x)
        out.append((u_seq.copy(), opt.copy()))
        x = x + 0.002 * (i + 1)
    used = c._npdev
    hits = c._npre_used
    c.close()
    return out, np.random.get_state(), used, hits


def test_controller_device_draw_equals_host_draw():
    """The drop-in with its default noise: the device draw gives the host draw's steps bit for bit and leaves
    np.random where the host draw (NumPy's values and state, tests/test_hostrng.py) leaves it."""
    a, st_a, used, hits = _loop(True)
    b, st_b, _, _ = _loop(False)
    assert used, "the controller did not take the device draw"
    assert hits == 3, "calls 2-4 use the draw queued by the call before"
    for (ua, oa), (ub, ob) in zip(a, b):
        np.testing.assert_array_equal(ua, ub)
        np.testing.assert_array_equal(oa, ob)
    assert _same_state(st_a, st_b)


def test_controller_device_draw_general_sigma():
    """A Sigma whose transform is a full 2 x 2 matrix (the sigma_k128_t20 fixture's [[20, 6], [6, 12]]) stays on
    the device draw: the host draw's steps and RNG state bit for bit, the queued draw used."""
    sig = SIGMAS["general"]
    a, st_a, used, hits = _loop(True, sigma=sig)
    b, st_b, _, _ = _loop(False, sigma=sig)
    assert used, "the controller did not take the device draw"
    assert hits == 3
    for (ua, oa), (ub, ob) in zip(a, b):
        np.testing.assert_array_equal(ua, ub)
        np.testing.assert_array_equal(oa, ob)
    assert _same_state(st_a, st_b)


def test_queued_draw_is_dropped_when_numpy_state_or_sigma_changes():
    """The draw queued for the next call is used only when np.random is still where the last call left it and
    Sigma's transform is unchanged: the caller's own draws, a reseed and a new Sigma between calls give the host
    draw's steps and state bit for bit."""
    def between(i, c):
        if i == 1:
            np.random.rand(3)                               # the caller consumes the stream
        elif i == 3:
            np.random.seed(7)
        elif i == 5:
            c.Sigma = np.eye(2) * 10.0                      # another plan
    a, st_a, used, hits = _loop(True, ticks=7, between=between)
    b, st_b, _, _ = _loop(False, ticks=7, between=between)
    assert used
    assert hits == 3, "used at calls 3, 5 and 7 only"
    for (ua, oa), (ub, ob) in zip(a, b):
        np.testing.assert_array_equal(ua, ub)
        np.testing.assert_array_equal(oa, ob)
    assert _same_state(st_a, st_b)


def _chain_loop(device_draw: bool, lam: float, ticks=3, K=4096, T=16):
    from mppi_robotarm_amd.chain import CHAIN7_X0, ChainMPPIController, gravity_torque
    from conftest import load_paths
    c = ChainMPPIController(0.006, load_paths()["xydq_circle"], T, K, param_lambda=lam, device=0,
                            u_init=gravity_torque(CHAIN7_X0[:7]), numpy_noise_on_device=device_draw)
    np.random.seed(4)
    out, precs, first = [], [], []
    for i in range(ticks):
        c.prev_waypoints_idx = 0
        first.append("f64" if c._spread else "f32")   # the engine this call's draw goes to first
        u0, u_seq, opt, _ = c.calc_control_input(CHAIN7_X0)
        out.append((u_seq.copy(), opt.copy()))
        precs.append(c.last_precision)
    used, hits = c._npdev, c._npre_used
    c.close()
    # the draw a call queues goes to that call's first engine; the next call uses it when its own first engine is
    # the same one (precision="auto" switches engines when the weights spread or stop spreading)
    want = sum(first[i] == first[i - 1] for i in range(1, ticks))
    return out, np.random.get_state(), used, precs, (hits, want)


@pytest.mark.parametrize("lam", [100.0, 3.0e5])
def test_chain_controller_device_draw_equals_host_draw(lam):
    """The 7-link drop-in's default noise on the device: the host draw's steps bit for bit; at lambda = 3e5 the
    weights spread and precision="auto" re-runs each step in fp64 on the other engine (the draw copied into its
    noise buffer)."""
    a, st_a, used, precs, (hits, want) = _chain_loop(True, lam)
    b, st_b, _, precs_b, _ = _chain_loop(False, lam)
    assert used, "the chain controller did not take the device draw"
    assert hits == want, "every call whose first engine is the last call's uses the draw queued beside that step"
    assert precs == precs_b
    assert lam < 1e4 or "f64" in precs
    for (ua, oa), (ub, ob) in zip(a, b):
        np.testing.assert_array_equal(ua, ub)
        np.testing.assert_array_equal(oa, ob)
    assert _same_state(st_a, st_b)
