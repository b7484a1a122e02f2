"""The vectorised Philox4x32-10 and the process-noise normals the GPU noise test checks
against (oracle.philox_np / oracle.noise_normals), on the host: philox_np equals the C
restatement orc_philox4x32_10 (itself pinned to the device by the bit-exact reset
draws, tests/test_gpu_parity.py) word for word."""
import numpy as np


def test_philox_np_equals_c(orc):
    rng = np.random.default_rng(0)
    C = rng.integers(0, 2 ** 32, (4, 300), dtype=np.uint64)
    for k in range(3):
        key = [int(v) for v in rng.integers(0, 2 ** 32, 2)]
        got = orc.philox_np(C, key)
        for i in range(0, 300, 7):
            want = orc.philox([int(C[j, i]) for j in range(4)], key)
            assert [int(got[j][i]) for j in range(4)] == want


def test_noise_normals_shape_and_range(orc):
    z = orc.noise_normals(3, np.arange(1 << 16), 1)
    assert z.shape == (1 << 16, 3)
    assert np.abs(z).max() <= np.sqrt(-2 * np.log(2.0 ** -24)) + 1e-9  # 24-bit u1 bound
    assert abs(z.mean()) < 0.02 and abs(z.std() - 1) < 0.02
    # keyed by (seed, gid, tick): another tick is another draw
    assert not np.array_equal(z, orc.noise_normals(3, np.arange(1 << 16), 2))
