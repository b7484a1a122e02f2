"""Every launcher branch of the policy-in-the-loop kernels, each with a
GPU case at a size that forces it and an assertion that the launcher chose it
(lz_get_launch_shape, the launchers' own decision functions: lz_internal.h
policy_shape / f32_policy_shape / attn_policy_shape / attn_f32_policy_shape).  The
round-3 race (DESIGN §5 "Round 3c") lived in a rollout branch no test reached at its
size; this file is the policy kernels' branch table.

Per case: the env part of the collect is bit-exact against lz_rollout fed the policy's
own clipped actions (observations, rewards, dones, the compact done list, the final
state), and the forward is checked on every recorded row --
  * float32 kernels: bit for bit vs oracle.mlp_f32 / oracle.attn_f32 of the input the
    kernel recorded (deterministic actions = the mean, values, last values);
  * bf16 kernels: vs the torch restatements with the same bf16 roundings (policy.
    reference_forward_*_bf16) within the tolerance of tests/test_gpu_policy.py, and
    the three bf16 MLP shapes are bit-identical to one another.

Branches (MI355X: 256 CUs):
  f32 MlpPolicy   split actor/critic waves (tiles < 8 x CUs): n < 32, ragged, grid-stride;
                  one wave per tile, 8 waves: exact fit, grid-stride + ragged; 4 waves
                  (variant bit 8192)
  f32 SB3-exact   per-step kernel, 4 waves / 8 waves + grid-stride
  bf16 MlpPolicy  interleaved nets + pipelined weights / interleaved / serial 32-env waves
                  (variant bits 128, 32) / serial 32-env x 8 grid-stride / 64-env waves
                  grid-stride + ragged
  bf16 attention  32-env waves x 4, grid-stride; LayerNorm + VecFrameStack(4 / 1)
  f32 attention   16-env waves x 8: n < 16, ragged, grid-stride; LayerNorm + stack(4)
                  grid-stride + ragged
"""
import numpy as np
import pytest
import torch

from conftest import bits_equal

pytestmark = pytest.mark.gpu

F32_MLP, F32_STEP, BF16_MLP, BF16_ATTN, BF16_LN, F32_ATTN, F32_LN = (
    "f32_mlp", "f32_step", "bf16_mlp", "bf16_attn", "bf16_ln", "f32_attn", "f32_ln")


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


def _mlp_sd(pol, O, A, seed, scale=0.4):
    net = pol.ActorCriticMlp(O, A, seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for p in net.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * (scale if p.dim() > 1 else 0.3))
    return {k: v.detach().clone() for k, v in net.state_dict().items()}


def _attn_sd(pol, I, A, seed, ln=False, scale=0.2):
    net = pol.ActorCriticAttn(I, A, seed=seed, layer_norm=ln)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for name, p in net.named_parameters():
            if "layer_norm" in name:
                p.copy_((1.0 if name.endswith("weight") else 0.0) + 0.2 * torch.randn(p.shape, generator=g))
            else:
                p.copy_(torch.randn(p.shape, generator=g) * (scale if p.dim() > 1 else 0.3))
    return {k: v.detach().clone() for k, v in net.state_dict().items()}


# (kind, system, n, K, variant, n_stack, expected kernel, grid_stride)
CASES = [
    (F32_MLP, "pmsm", 20, 4, 0, 1, "policy_split", False),         # n < 32: one partial tile
    (F32_MLP, "pmsm", 1000, 6, 0, 1, "policy_split", False),       # ragged last tile
    (F32_MLP, "lorenz3", 40001, 3, 0, 1, "policy_split", True),    # 313 groups on 256 CUs
    (F32_MLP, "pmsm", 65536, 3, 0, 1, "policy", False),            # 8 waves, 256 groups exactly
    (F32_MLP, "hr", 70001, 3, 0, 1, "policy", True),               # 8 waves, grid-stride, ragged
    (F32_MLP, "pmsm", 1000, 4, 8192, 1, "policy", False),          # 4 waves, one per tile
    (F32_STEP, "pmsm", 1000, 4, 0, 1, "policy_step", False),       # 4 waves
    (F32_STEP, "lorenz4", 70001, 3, 0, 1, "policy_step", True),    # 8 waves, grid-stride
    (BF16_MLP, "pmsm", 1000, 5, 0, 1, "policy_pair_pipe", False),  # nets interleaved, pipelined
    (BF16_MLP, "pmsm", 1000, 5, 128, 1, "policy_pair", False),     # interleaved
    (BF16_MLP, "pmsm", 1000, 5, 32, 1, "policy", False),           # serial 32-env waves x 8
    (BF16_MLP, "lorenz3", 70000, 3, 0, 1, "policy", True),         # serial x 8, grid-stride
    (BF16_MLP, "pmsm", 262147, 3, 0, 1, "policy", True),           # 64-env waves, ragged
    (BF16_ATTN, "hr", 1000, 4, 0, 1, "policy_attn", False),
    (BF16_ATTN, "hr", 40000, 3, 0, 1, "policy_attn", True),
    (BF16_LN, "hr", 1000, 4, 0, 4, "policy_attn", False),
    (BF16_LN, "hr", 40001, 3, 0, 1, "policy_attn", True),
    (F32_ATTN, "hr", 5, 4, 0, 1, "policy_attn_f32", False),        # n < 16
    (F32_ATTN, "pmsm", 1000, 4, 0, 1, "policy_attn_f32", False),   # ragged
    (F32_ATTN, "hr", 40000, 3, 0, 1, "policy_attn_f32", True),     # 313 groups
    (F32_LN, "hr", 1000, 4, 0, 4, "policy_attn_f32", False),
    (F32_LN, "hr", 33001, 3, 0, 4, "policy_attn_f32", True),       # 258 groups, ragged
]
CALL = {F32_MLP: 3, F32_STEP: 4, BF16_MLP: 2, BF16_ATTN: 5, BF16_LN: 6, F32_ATTN: 7, F32_LN: 8}


def _collector(gl, pol, kind, system, n, variant, n_stack, seed=5):
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    kw = dict(max_episode_steps=3)
    if system in ("pmsm", "hr"):
        kw["add_noise"] = True
    envp = gl.BatchedEnv(system, n, seed=seed, variant=variant, **kw)
    envr = gl.BatchedEnv(system, n, seed=seed, **kw)
    O, A = envp.obs_dim, envp.action_dim
    f32 = kind in (F32_MLP, F32_STEP, F32_ATTN, F32_LN)
    ln = kind in (BF16_LN, F32_LN)
    if kind in (F32_MLP, F32_STEP, BF16_MLP):
        sd = _mlp_sd(pol, O, A, seed=7, scale=0.2 if kind == BF16_MLP else 0.4)
    else:
        sd = _attn_sd(pol, n_stack * O if ln else O, A, seed=3, ln=ln)
    rms = None
    if kind == F32_STEP:  # SB3-exact VecNormalize: one launch per step
        rms = DeviceRunningMeanStd(O, envp.device)
    col = pol.FusedRolloutCollector(envp, sd, bootstrap=False, deterministic=True, obs_rms=rms,
                                    training=True, capture_terminal=4 * n, frame_stack=n_stack if ln else 1,
                                    precision="fp32" if f32 else "bf16")
    if kind == F32_STEP:
        assert col.per_step_vecnorm
    return envp, envr, col, sd, O, A


@pytest.mark.parametrize("kind,system,n,K,variant,n_stack,kernel,stride", CASES)
def test_policy_branch(gl, pol, orc, kind, system, n, K, variant, n_stack, kernel, stride):
    from gym_lorenz import _native as nat

    envp, envr, col, sd, O, A = _collector(gl, pol, kind, system, n, variant, n_stack)
    sh = nat.launch_shape(envp._h, CALL[kind])
    assert sh["kernel"] == kernel, sh
    assert sh["grid_stride"] == stride, sh
    assert sh["grid"] <= sh["groups"] and (stride or sh["grid"] == sh["groups"]), sh
    obs0 = _np(col.reset())
    assert np.array_equal(obs0, _np(envr.reset()))
    b = col.collect(K)
    lo, hi = pol.action_bounds(system)
    acts = torch.clamp(b.actions, lo, hi).contiguous()
    obs_r, rew_r, done_r, (didx, tobs, nd) = envr.rollout(acts, capture_terminal=4 * n)
    # env part: bit-exact
    assert torch.equal(b.dones, done_r)
    assert torch.equal(b.rewards, rew_r)  # no bootstrap
    assert torch.equal(b.last_obs.view(torch.int32), obs_r[-1].view(torch.int32))
    m = int(nd.item())
    assert m > 0 and int(b.n_done.item()) == m
    o1, o2 = np.argsort(_np(b.done_idx[:m])), np.argsort(_np(didx[:m]))
    assert np.array_equal(_np(b.done_idx[:m])[o1], _np(didx[:m])[o2])
    assert bits_equal(_np(b.terminal_obs[:m])[o1], _np(tobs[:m])[o2])
    for p in range(3):
        assert torch.equal(envp.get_state(p), envr.get_state(p))
    # forward on every recorded row
    I = b.observations.shape[-1]
    x = _np(b.observations).reshape(-1, I)
    act = _np(b.actions).reshape(-1, A)
    val = _np(b.values).reshape(-1)
    if kind in (F32_MLP, F32_STEP):
        mref, vref = orc.mlp_f32(sd, x)
    elif kind in (F32_ATTN, F32_LN):
        mref, vref = orc.attn_f32(sd, x)
    if kind in (F32_MLP, F32_STEP, F32_ATTN, F32_LN):
        assert bits_equal(act, mref), np.nanmax(np.abs(act - mref))
        assert bits_equal(val, vref), np.nanmax(np.abs(val - vref))
    else:
        ref = {BF16_MLP: pol.reference_forward_bf16, BF16_ATTN: pol.reference_forward_attn_bf16,
               BF16_LN: pol.reference_forward_attn_ln_bf16}[kind]
        mt, vt = ref(sd, torch.from_numpy(x))
        f = np.isfinite(x).all(1)
        tol = 2e-2 if kind == BF16_MLP else 3e-2
        np.testing.assert_allclose(act[f], _np(mt)[f], atol=tol, rtol=tol)
        np.testing.assert_allclose(val[f], _np(vt)[f], atol=tol, rtol=tol)
        assert np.median(np.abs(val[f] - _np(vt)[f])) < 2e-3
    envp.close()
    envr.close()


def test_bf16_mlp_shapes_bit_identical(gl, pol):
    """The bf16 MlpPolicy shapes reachable at one size (interleaved + pipelined,
    interleaved, serial 32-env waves) give bit-identical collects."""
    outs = []
    for var in (0, 128, 32):
        envp, _, col, _, _, _ = _collector(gl, pol, BF16_MLP, "pmsm", 1000, var, 1, seed=9)
        col.reset()
        outs.append(col.collect(5))
        envp.close()
    for b in outs[1:]:
        for f in ("observations", "actions", "log_probs", "values", "rewards", "dones", "last_values"):
            assert torch.equal(getattr(b, f), getattr(outs[0], f)), f


@pytest.mark.parametrize("system,n,variant,kernel,no_done", [
    ("lorenz3", 16384, 0, "rollout_wave", False),    # one-wave, below 32,768: no split
    ("lorenz3", 32768, 0, "rollout_split", True),    # two lanes per env, done-free (no TimeLimit)
    ("lorenz3", 65536, 0, "rollout", True),          # 256-lane from 256 x CUs
    ("lorenz3", 32768, 2048, "rollout_split", False),  # variant 2048: the done path
    ("lorenz4", 49152, 0, "rollout", False),         # LORENZ4 f32: 256-lane from 3/4 x 256 x CUs
    ("lorenz4", 40960, 0, "rollout_wave", False),
    ("pmsm", 100000, 0, "rollout_wave", False),      # PMSM / HR: one-wave below 131,072
    ("pmsm", 32768, 0, "rollout_pair", False),       # PMSM: lane pairs at 2 < waves / CU <= 4
    ("pmsm", 16385, 0, "rollout_pair", False),
    ("pmsm", 16384, 0, "rollout_wave", False),
    ("pmsm", 32769, 0, "rollout_wave", False),
    ("pmsm", 200000, 1 << 27, "rollout_pair", False),  # forced at any N
    ("pmsm", 4097, 1 << 28, "rollout_wave", False),    # disabled
    ("hr", 32768, 0, "rollout_wave", False),          # (HR has no lane-pair step)
    ("hr", 131072, 0, "rollout", False),
])
def test_env_rollout_branch_reported(gl, system, n, variant, kernel, no_done):
    """lz_get_launch_shape reports the rollout branch launch_rollout_d takes (the
    rollout == steps cases of test_gpu_parity.py cover each branch's arithmetic)."""
    from gym_lorenz import _native as nat

    kw = {"add_noise": True} if system in ("pmsm", "hr") else {}
    be = gl.BatchedEnv(system, n, seed=1, variant=variant, **kw)
    sh = nat.launch_shape(be._h, nat.CALL_ROLLOUT)
    assert sh["kernel"] == kernel and sh["no_done"] == no_done, sh
    st = nat.launch_shape(be._h, nat.CALL_STEP)
    assert st["kernel"] in ("step", "step_multi") and st["envs_per_wave"] == 64
    be.close()
