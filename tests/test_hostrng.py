"""The drop-in's NumPy-stream noise (control.py:154-164): hostrng.multivariate_normal, whose standard-normal
stream is threaded in C (csrc/np_legacy_gauss.c), equals np.random.multivariate_normal value for value and
leaves the global RNG in the state NumPy leaves (the next draws agree too)."""
import os

import numpy as np
import pytest

from mppi_robotarm_amd import hostrng
from mppi_robotarm_amd.build import build_host_rng

build_host_rng()   # gcc, under a second; a no-op when the library is current


def _state_eq(a, b):
    return a[0] == b[0] and np.array_equal(a[1], b[1]) and a[2] == b[2] and a[3] == b[3] and a[4] == b[4]


def test_library_is_built_and_used():
    np.random.seed(5)
    assert hostrng.legacy_standard_normal(1 << 16) is not None


@pytest.mark.parametrize("seed,size,cov", [
    (0, (16384, 64), np.eye(2) * 20.0),                       # run.py's Sigma
    (3, (4097, 31), np.array([[20.0, 5.0], [5.0, 10.0]])),    # non-diagonal, odd count of pairs
    (7, (20001, 3), np.eye(7) * 3.0 + 0.5),                   # the 7-link chain's dimension, odd total
    (11, (1 << 15, 1), np.eye(1) * 2.0),
    (13, (1000, 7), np.eye(2)),                               # below the threshold: NumPy itself
])
@pytest.mark.parametrize("pre", [0, 1, 1001])                 # stream position; an odd pre leaves a cached Gaussian
def test_equals_numpy_multivariate_normal(seed, size, cov, pre):
    mu = np.zeros(cov.shape[0])
    np.random.seed(seed)
    np.random.standard_normal(pre)
    a = np.random.multivariate_normal(mu, cov, size)
    sa = np.random.get_state()
    na = np.random.standard_normal(5)
    np.random.seed(seed)
    np.random.standard_normal(pre)
    b = hostrng.multivariate_normal(mu, cov, size)
    sb = np.random.get_state()
    nb = np.random.standard_normal(5)
    assert a.shape == b.shape and a.dtype == b.dtype
    assert np.array_equal(a, b)
    assert _state_eq(sa, sb)
    assert np.array_equal(na, nb)


def test_state_at_block_boundaries_and_retry_sizes():
    """Positions at 0 / 623 / 624 within the key array and draws that end at every parity."""
    for pos_skip in (0, 623, 624, 1248):
        for n in (1 << 15, (1 << 15) + 1, (1 << 15) + 2, 100003):
            np.random.seed(17)
            np.random.randint(0, 2**31, size=pos_skip, dtype=np.int64)   # advance the word position
            s0 = np.random.get_state()
            a = np.random.standard_normal(n)
            sa = np.random.get_state()
            np.random.set_state(s0)
            b = hostrng.legacy_standard_normal(n)
            assert b is not None and np.array_equal(a, b)
            assert _state_eq(sa, np.random.get_state())


def test_errors_are_numpys():
    with pytest.raises(ValueError):
        hostrng.multivariate_normal(np.zeros(2), np.eye(3), (40000, 2))
    with pytest.warns(RuntimeWarning):
        hostrng.multivariate_normal(np.zeros(2), np.array([[1.0, 2.0], [0.0, 1.0]]), (40000, 2))


def _jump_lib():
    import ctypes as C
    lib = hostrng._load()
    lib.mppi_np_jump_config.restype = C.c_int
    lib.mppi_np_jump_config.argtypes = [C.c_int]
    return lib


def test_jump_ahead_self_test_passes():
    """The twist in parallel rests on MT19937's jump-ahead: the characteristic polynomial found by
    Berlekamp-Massey (degree 19937, 135 terms) and two jumps checked against the sequential twist."""
    assert _jump_lib().mppi_np_jump_config(0) == 1


@pytest.mark.parametrize("pre", [0, 5, 1001])
@pytest.mark.parametrize("n", [1 << 15, 300001, 2_000_000])
def test_parallel_twist_equals_numpy(n, pre):
    """The threads' ranges start at jumped blocks (the threshold lowered to 8 blocks so that every size here
    takes that path): values and the state left behind equal NumPy's."""
    lib = _jump_lib()
    lib.mppi_np_jump_config(8)
    try:
        np.random.seed(23 + pre)
        np.random.standard_normal(pre)
        s0 = np.random.get_state()
        a = np.random.standard_normal(n)
        sa = np.random.get_state()
        np.random.set_state(s0)
        b = hostrng.legacy_standard_normal(n)
        assert b is not None and np.array_equal(a, b)
        assert _state_eq(sa, np.random.get_state())
    finally:
        lib.mppi_np_jump_config(4096)


@pytest.mark.parametrize("cov", [np.eye(2) * 20.0, np.diag([1.0, 5.0]), np.diag([20.0, 16, 12, 8, 4, 2, 1]),
                                 np.array([[0.0, 0.0], [0.0, 3.0]])])
def test_std_noise_equals_numpy(cov):
    """multivariate_normal_std: the standard normals into the caller's buffer plus a scaled column
    permutation (a diagonal Sigma, sorted or not) give NumPy's values exactly and leave its state; a Sigma
    whose transform mixes columns draws nothing."""
    d = cov.shape[0]
    size = (9001, 5)
    np.random.seed(31)
    a = np.random.multivariate_normal(np.zeros(d), cov, size)
    sa = np.random.get_state()
    np.random.seed(31)
    buf = np.empty(9001 * 5 * d + 3)
    r = hostrng.multivariate_normal_std(np.zeros(d), cov, size, buf)
    assert r is not None and np.shares_memory(r.z, buf)
    x = r.z[..., r.src] * r.scale + r.mean
    assert np.array_equal(a, x) and _state_eq(sa, np.random.get_state())
    assert r.eps(3, 4, d - 1) == a[3, 4, d - 1]
    np.random.seed(31)
    s0 = np.random.get_state()
    assert hostrng.multivariate_normal_std(np.zeros(2), np.array([[20.0, 5.0], [5.0, 10.0]]), size, buf) is None
    assert _state_eq(s0, np.random.get_state())


# ---------------------------------------------------------------- the device draw's host inputs

def test_log_replica_equals_libm_log():
    """csrc/np_glibc_log.h on the constants read from libm (hostrng.log_params) equals libm's log() -- the log
    NumPy's legacy_gauss calls -- bit for bit: random values over (0, 1), the near-1 branch and both its
    edges, the smallest r2 an accepted polar attempt can have, powers of two and their neighbours."""
    D = hostrng.log_params()
    assert D is not None and D.shape == (274,)
    lib = hostrng._load()
    rng = np.random.default_rng(0)
    lo, hi = 1.0 - 2.0 ** -4, 1.0 + float.fromhex("0x1.09p-4")
    edges = [np.nextafter(lo, 0), lo, np.nextafter(lo, 2), np.nextafter(1.0, 0), 1.0, np.nextafter(hi, 0), hi,
             np.nextafter(hi, 2), 2.0 ** -104, 2.0 ** -52, 0.5, np.nextafter(0.5, 0), np.nextafter(0.5, 1)]
    pw = 2.0 ** -np.arange(1, 105)
    x = np.concatenate([rng.random(2_000_000), lo + rng.random(500_000) * (1 - lo), np.array(edges), pw,
                        np.nextafter(pw, 0), np.nextafter(pw, 1)])
    x = np.ascontiguousarray(x[(x > 0) & (x <= 1)])
    assert lib.mppi_np_log_mismatches(D.ctypes.data, x.ctypes.data, x.size) == 0


def _mt_blocks(key, nblk):
    """nblk key arrays from `key` by NumPy's twist (vectorised over the three in-place phases)."""
    out = np.empty((nblk, 624), dtype=np.uint32)
    out[0] = key
    A, UP, LO = np.uint32(0x9908b0df), np.uint32(0x80000000), np.uint32(0x7fffffff)

    def mix(a, b):
        y = (a & UP) | (b & LO)
        return (y >> np.uint32(1)) ^ ((np.uint32(0) - (y & np.uint32(1))) & A)
    for b in range(1, nblk):
        o, k = out[b - 1], out[b]
        k[:227] = o[397:624] ^ mix(o[:227], o[1:228])
        k[227:454] = k[0:227] ^ mix(o[227:454], o[228:455])
        k[454:623] = k[227:396] ^ mix(o[454:623], o[455:624])
        k[623] = k[396] ^ mix(o[623:624], k[0:1])[0]
    return out


@pytest.mark.parametrize("P,s", [(64, 1), (64, 3), (512, 2)])
def test_jump_polynomials_reach_the_stream_starts(P, s):
    """hostrng.jump_polys: the window form of the jump (the XOR of the word sequence's windows at the
    polynomial's set bits, as np_jump_kernel evaluates it) then one twist gives key array P s exactly -- the
    generator streams' starting blocks of the device draw."""
    np.random.seed(17)
    key = np.random.get_state()[1].astype(np.uint32)
    nblk = P * s + 1
    blocks = _mt_blocks(key, max(nblk, 35))
    poly = hostrng.jump_polys(P, s + 1)[s - 1]
    bits = np.nonzero(np.unpackbits(poly.view(np.uint8), bitorder="little"))[0]
    assert bits.max() < 19937
    seq = blocks[:35].reshape(-1)
    jumped = np.zeros(624, dtype=np.uint32)
    for d in bits:
        jumped ^= seq[d:d + 624]
    nxt = _mt_blocks(jumped, 2)[1]
    np.testing.assert_array_equal(nxt, blocks[P * s])


@pytest.mark.parametrize("cov", [[[20.0, 6.0], [6.0, 12.0]], [[2.0, -1.5], [-1.5, 3.0]], [[1.0, 0.999], [0.999, 1.0]]])
def test_dot2_model_pins_numpys_rounding(cov):
    """The device draw's general 2 x 2 transform (mppi_np_target.dot2): on this host np.dot(z, m) of
    multivariate_normal's matrix equals fma(z1, m[1, j], z0 * m[0, j]) bit for bit (hostrng.dot2_model, checked
    again at run time wherever the draw runs), and device_plan hands that matrix over; a diagonal Sigma keeps the
    scaled column permutation."""
    cov = np.array(cov)
    u, s, v = np.linalg.svd(cov)
    m = np.sqrt(s)[:, None] * v
    assert hostrng.dot2_model(m)
    plan = hostrng.device_plan(np.zeros(2), cov)
    assert plan is not None and plan[4] is not None and np.array_equal(plan[4], m)
    # the reference's own draw reproduced with the model on NumPy's standard normals
    np.random.seed(3)
    want = np.random.multivariate_normal(np.zeros(2), cov, (50, 7))
    np.random.seed(3)
    z = np.random.standard_normal((50 * 7, 2))
    got = np.empty_like(z)
    hostrng._load().mppi_np_dot2_fma(z.ctypes.data, z.shape[0], np.ascontiguousarray(m).ctypes.data, got.ctypes.data)
    got += 0.0
    np.testing.assert_array_equal(got.reshape(50, 7, 2), want)
    diag = hostrng.device_plan(np.zeros(2), np.eye(2) * 20.0)
    assert diag is not None and diag[4] is None

