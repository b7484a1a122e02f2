"""The policy blob's format tag on the GPU (include/lorenz_env.h LZ_BLOB_*).

A float32 and an i8x4 blob of one family have the same size and offsets; only the launch's
LZ_POLICY_I8X4 flag (and the entry point) says how to read one.  Every float32 / i8x4
policy kernel compares the packer's tag with the format its launch expects and, on a
mismatch, runs on an all-NaN copy of the blob.  Here each kernel family gets the OTHER
precision's blob swapped in behind the collector's host check: every action, log-prob,
value, reward and last value the launch writes is NaN (not a rollout on misread
weights); the correctly tagged blob gives finite outputs on the same handle."""
import numpy as np
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.filterwarnings("ignore::RuntimeWarning")]


@pytest.fixture(scope="module")
def gl():
    import gym_lorenz

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return gym_lorenz


@pytest.fixture(scope="module")
def pol():
    from gym_lorenz import policy

    return policy


def _np(t):
    return t.detach().cpu().numpy()


def _outputs(b):
    return {f: _np(getattr(b, f)) for f in ("actions", "log_probs", "values", "rewards",
                                            "last_values")}


def _run(gl, pol, system, n, sd, precision, swap, variant=0, frame_stack=1, vn=None, **ekw):
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    env = gl.BatchedEnv(system, n, seed=3, variant=variant, **ekw)
    rms = None
    if vn is not None:
        rms = DeviceRunningMeanStd(env.obs_dim, env.device)
    col = pol.FusedRolloutCollector(env, sd, bootstrap=False, obs_rms=rms, training=vn is not None,
                                    precision=precision, frame_stack=frame_stack,
                                    vecnorm_update=vn)
    if swap is not None:  # the other precision's blob, behind the host-side tag check
        col.blob = torch.from_numpy(swap).to(env.device)
    col.reset()
    out = _outputs(col.collect(4))
    env.close()
    return out


def _all_nan(out):
    for k, v in out.items():
        assert np.isnan(v).all(), "%s: %d finite of %d" % (k, np.isfinite(v).sum(), v.size)


def _all_finite(out):
    for k, v in out.items():
        assert np.isfinite(v).all(), k


@pytest.mark.parametrize("variant", [0, 8192])  # split kernel / one-wave kernel
@pytest.mark.parametrize("launch", ["fp32", "i8x4"])
def test_mlp_blob_flag_mismatch_is_nan(gl, pol, variant, launch):
    sd = pol.ActorCriticMlp(6, 2, seed=4).state_dict()
    other = pol.pack_policy_i8x4(sd, 6, 2) if launch == "fp32" else pol.pack_policy_f32(sd, 6, 2)
    _all_nan(_run(gl, pol, "pmsm", 4099, sd, launch, other, variant, add_noise=True,
                  vn="rollout" if launch == "i8x4" else None))
    _all_finite(_run(gl, pol, "pmsm", 4099, sd, launch, None, variant, add_noise=True,
                     vn="rollout" if launch == "i8x4" else None))


def test_policy_step_f32_refuses_an_i8x4_blob(gl, pol):
    """lz_policy_step_f32 (SB3-order VecNormalize collect) reads float32 blobs only."""
    sd = pol.ActorCriticMlp(6, 2, seed=4).state_dict()
    _all_nan(_run(gl, pol, "pmsm", 2051, sd, "fp32", pol.pack_policy_i8x4(sd, 6, 2),
                  vn="step", add_noise=True))
    _all_finite(_run(gl, pol, "pmsm", 2051, sd, "fp32", None, vn="step", add_noise=True))


@pytest.mark.parametrize("launch", ["fp32", "i8x4"])
def test_attention_blob_flag_mismatch_is_nan(gl, pol, launch):
    sd = pol.ActorCriticAttn(6, 2, seed=4).state_dict()
    other = (pol.pack_attn_policy_i8x4(sd, 6, 2) if launch == "fp32"
             else pol.pack_attn_policy_f32(sd, 6, 2))
    _all_nan(_run(gl, pol, "hr", 2053, sd, launch, other, add_noise=True))
    _all_finite(_run(gl, pol, "hr", 2053, sd, launch, None, add_noise=True))


def test_attention_ln_entry_refuses_a_plain_attention_blob(gl, pol):
    """The LayerNorm entry (frame-stacked) with the plain extractor's blob, and i8x4 LN
    with the float32 LN blob."""
    sd = pol.ActorCriticAttn(24, 2, seed=4, layer_norm=True).state_dict()
    sd_plain = pol.ActorCriticAttn(6, 2, seed=4).state_dict()
    plain = pol.pack_attn_policy_f32(sd_plain, 6, 2)
    _all_nan(_run(gl, pol, "hr", 2053, sd, "fp32", plain, frame_stack=4, add_noise=True))
    _all_nan(_run(gl, pol, "hr", 2053, sd, "i8x4", pol.pack_attn_ln_policy_f32(sd, 24, 2),
                  frame_stack=4, add_noise=True))
    _all_finite(_run(gl, pol, "hr", 2053, sd, "i8x4", None, frame_stack=4, add_noise=True))
