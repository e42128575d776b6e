"""The device noise stream, element by element (noise="device", SURVEY §8 f1;
the on-device alternative to _calc_epsilon, control.py:154-164).  Each element
of philox_noise_kernel / chain_philox_kernel must equal the host restatement
oracle/philox_ref.py (standard Philox4x32-10, pinned by Random123's known
answers in tests/test_philox_ref.py) at the same (seed, step, t, global k, d):
for odd T (the last step pair is half used), ragged K (partial workgroups),
nonzero shard offsets and seeds / steps with high 32-bit words.  The tolerance
covers only the fp32 transcendentals / Cholesky of the device's Box-Muller
against the host's fp64 (a wrong counter or word mapping gives O(1) errors).
The device evaluates Box-Muller on the hardware transcendentals (v_log_f32,
v_sqrt_f32, v_sin_f32 / v_cos_f32 in revolutions); the bench's own stream
(K = 65536, T = 64, 4.2 M elements) is checked whole, so the rare draws with
u0 near 1, where the log's absolute error matters most, are in it."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import philox_ref as P  # noqa: E402
from conftest import record  # noqa: E402

TOL = 2e-5


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


@pytest.mark.parametrize("K_local,T,k_offset,seed,step", [(1000, 7, 0, 42, 3), (777, 1, 5000, 2 ** 40 + 9, 2 ** 33 + 1),
                                                          (4099, 16, 123456, 0, 0), (65536, 64, 0, 1234, 0)])
def test_arm_noise_stream(K_local, T, k_offset, seed, step):
    from mppi_robotarm_amd.engine import RolloutEngine
    from mppi_robotarm_amd.params import ArmParams
    sig = np.array([[20.0, 6.0], [6.0, 12.0]])
    eng = RolloutEngine(K_local, T, 0.006, 100.0, 0.98, sig, [0.5, 0.5, 5, 5], [5, 5, 50, 50], 0.0, ArmParams(),
                        K_total=k_offset + K_local, k_offset=k_offset, device=0)
    dev = eng.philox_noise(seed, step).double().cpu().numpy()
    ref = P.arm_noise(K_local, T, k_offset, seed, step, sig)
    err = np.abs(dev - ref) / (1.0 + np.abs(ref))
    record("philox_stream", K=K_local, T=T, max_err=float(np.max(err)), p99_err=float(np.percentile(err, 99)))
    assert float(np.max(err)) < TOL, float(np.max(err))
    eng.close()


@pytest.mark.parametrize("K_local,T,k_offset,seed,step", [(333, 5, 0, 7, 1), (1500, 3, 2048, 2 ** 35 + 3, 2 ** 32 + 5)])
def test_chain_noise_stream(K_local, T, k_offset, seed, step):
    from mppi_robotarm_amd.chain import CHAIN7_SIGMA, ChainEngine
    eng = ChainEngine(K_local, T, 0.006, 100.0, 0.98, CHAIN7_SIGMA, [0.5, 0.5, 5, 5], [5, 5, 50, 50],
                      K_total=k_offset + K_local, k_offset=k_offset, device=0)
    dev = eng.philox_noise(seed, step).double().cpu().numpy().transpose(0, 2, 1)   # device [T][K][n] -> (T, n, K)
    ref = P.chain_noise(K_local, T, 7, k_offset, seed, step, CHAIN7_SIGMA)
    err = np.abs(dev - ref) / (1.0 + np.abs(ref))
    assert float(np.max(err)) < TOL, float(np.max(err))
    eng.close()
