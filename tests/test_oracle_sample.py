"""The oracle on a SAMPLE of global env ids (oracle_tl.OracleTL gids=, used by the
max-size GPU cases) reproduces the same rows of a full-batch run bit for bit: the Philox
reset draws are keyed by (seed, global env id, tick), the step is per env."""
import numpy as np

from oracle_tl import OracleTL


def test_sampled_rows_equal_full_batch():
    import oracle as orc

    n, L = 4099, 3
    rng = np.random.default_rng(2)
    steps0 = rng.integers(0, L, n).astype(np.int32)
    gids = np.unique(np.concatenate([[0, 1, n - 1], rng.integers(0, n, 300)])).astype(np.int64)
    full = OracleTL(orc, "l3", np.float32, n, 9, L, steps0)
    part = OracleTL(orc, "l3", np.float32, gids.size, 9, L, steps0[gids], gids=gids)
    assert np.array_equal(full.st[gids].view(np.int32), part.st.view(np.int32))
    for k in range(7):
        a = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
        o, r, d, idx, term = full.step(a)
        po, pr, pd, pidx, pterm = part.step(a[gids])
        assert np.array_equal(o[gids].view(np.int32), po.view(np.int32)), k
        assert np.array_equal(r[gids].view(np.int32), pr.view(np.int32)), k
        assert np.array_equal(d[gids], pd), k
        sel = np.isin(idx, gids)
        assert np.array_equal(idx[sel], gids[pidx]), k
        assert np.array_equal(term[sel].view(np.int32), pterm.view(np.int32)), k
    assert np.array_equal(full.st[gids].view(np.int32), part.st.view(np.int32))
