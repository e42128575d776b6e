"""The host Philox restatement (oracle/philox_ref.py) against Random123's
published known-answer vectors for Philox4x32-10 (kat_vectors: philox4x32 10
rounds), so the GPU noise-stream test (tests/test_gpu_noise_stream.py) pins
the device generator to the standard algorithm, not merely to itself."""
import numpy as np

import philox_ref as P

KAT = [  # (ctr[4], key[2]) -> out[4]
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def test_philox4x32_10_known_answers():
    for ctr, key, want in KAT:
        got = tuple(int(x) for x in P.philox4x32_10(ctr, key))
        assert got == want, [hex(x) for x in got]


def test_noise_layout_and_moments():
    sig = np.array([[20.0, 6.0], [6.0, 12.0]])
    e = P.arm_noise(4000, 9, 123, 7, 2, sig)
    assert e.shape == (9, 4000, 2)
    np.testing.assert_allclose(np.cov(e.reshape(-1, 2).T), sig, rtol=0.05)
    # a shard's slice is the slice of the unsharded draw
    e2 = P.arm_noise(1000, 9, 123 + 2500, 7, 2, sig)
    np.testing.assert_array_equal(e2, e[:, 2500:3500])
    c = P.chain_noise(3000, 3, 7, 0, 5, 1, np.diag([20.0, 16, 12, 8, 4, 2, 1]))
    assert c.shape == (3, 7, 3000)
    np.testing.assert_allclose(c.var(axis=(0, 2)), [20.0, 16, 12, 8, 4, 2, 1], rtol=0.1)
