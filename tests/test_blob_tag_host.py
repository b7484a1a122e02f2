"""The policy blobs' format tag (include/lorenz_env.h LZ_BLOB_*): the float32
and i8x4 blobs of one family have the same size and offsets, so each packer writes a
16-byte tag that lz_policy_blob_format reads back and the kernels check against their
launch (a mismatch runs on an all-NaN blob copy: tests/test_gpu_blob_tag.py).  Host only."""
import numpy as np
import pytest

from gym_lorenz import _native as nat


@pytest.fixture(scope="module")
def pol():
    from gym_lorenz import policy

    return policy


def _fmt(blob):
    return int(nat.lib.lz_policy_blob_format(blob.ctypes.data, blob.size))


def test_every_packer_tags_its_format(pol):
    mlp = pol.ActorCriticMlp(6, 2, seed=1).state_dict()
    att = pol.ActorCriticAttn(6, 2, seed=1).state_dict()
    ln = pol.ActorCriticAttn(24, 2, seed=1, layer_norm=True).state_dict()
    cases = [(pol.pack_policy_f32(mlp, 6, 2), nat.BLOB_MLP_F32),
             (pol.pack_policy_i8x4(mlp, 6, 2), nat.BLOB_MLP_I8X4),
             (pol.pack_attn_policy_f32(att, 6, 2), nat.BLOB_ATTN_F32),
             (pol.pack_attn_policy_i8x4(att, 6, 2), nat.BLOB_ATTN_I8X4),
             (pol.pack_attn_ln_policy_f32(ln, 24, 2), nat.BLOB_ATTN_LN_F32),
             (pol.pack_attn_ln_policy_i8x4(ln, 24, 2), nat.BLOB_ATTN_LN_I8X4)]
    for blob, want in cases:
        assert _fmt(blob) == want
    # the collector's expectation per launch
    assert pol.blob_format(False, False, False) == nat.BLOB_MLP_F32
    assert pol.blob_format(True, False, True) == nat.BLOB_ATTN_I8X4
    assert pol.blob_format(True, True, False) == nat.BLOB_ATTN_LN_F32
    # the bf16 blobs carry no tag, nor does a zeroed / truncated / corrupted blob
    assert _fmt(pol.pack_policy(mlp, 6, 2)) == nat.BLOB_UNKNOWN
    b = cases[1][0].copy()
    assert _fmt(b[: b.size - 1]) == nat.BLOB_UNKNOWN
    assert _fmt(np.zeros_like(b)) == nat.BLOB_UNKNOWN
    assert nat.lib.lz_policy_blob_format(None, 1 << 20) == nat.BLOB_UNKNOWN
    c = cases[0][0]  # packing is deterministic
    assert np.array_equal(c, pol.pack_policy_f32(mlp, 6, 2))


def test_tag_bytes_are_where_the_header_says(pol):
    """kF32Tag = kF32HB + 48 in net 0; kAFTag = kAFPi + kAXTag (lz_internal.h)."""
    mlp = pol.ActorCriticMlp(6, 2, seed=1).state_dict()
    att = pol.ActorCriticAttn(6, 2, seed=1).state_dict()
    for blob, fmt in ((pol.pack_policy_f32(mlp, 6, 2), nat.BLOB_MLP_F32),
                      (pol.pack_attn_policy_f32(att, 6, 2), nat.BLOB_ATTN_F32)):
        w = np.frombuffer(blob.tobytes(), np.uint32)
        want = np.array([0x42505A4C, fmt, ~fmt & 0xFFFFFFFF, 0x42505A4C ^ fmt], np.uint32)
        hits = [i for i in range(w.size - 3) if np.array_equal(w[i: i + 4], want)]
        assert len(hits) == 1
        for j in range(16):  # flipping any tag byte unrecognises the blob
            c = blob.copy()
            c[4 * hits[0] + j] ^= 0x10
            assert _fmt(c) == nat.BLOB_UNKNOWN


def test_collector_refuses_a_mismatched_blob(pol, monkeypatch):
    """FusedRolloutCollector.set_params checks the packed blob's tag on the host before the
    upload (a packer bug, or a blob swapped in by hand, never reaches a launch)."""
    mlp = pol.ActorCriticMlp(6, 2, seed=1).state_dict()

    class Env:  # the collector needs only these before set_params packs
        num_envs, obs_dim, action_dim, system_name = 4, 6, 2, "pmsm"
        device = "cpu"

    monkeypatch.setattr(pol, "pack_policy_f32", pol.pack_policy_i8x4)  # a wrong packer
    col = pol.FusedRolloutCollector.__new__(pol.FusedRolloutCollector)
    col.env, col.precision, col.frame_stack, col.obs_rms = Env, "fp32", 1, None
    col.vecnorm_update, col.O, col.A, col.device, col.training = None, 6, 2, "cpu", True
    with pytest.raises(nat.LorenzEnvError):
        col.set_params(mlp)
