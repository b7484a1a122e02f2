"""The opt-in "i8x4" precision of the float32 MlpPolicy on the host (no GPU):
lz_policy_pack_i8x4's layer-2 digits and row shifts where mlp_i8_tail reads them, the
oracle (lz_oracle.c orc_mlp_i8x4) against float64 arithmetic and against the reference's
own eight trained PMSM policies, NaN propagation and the packer's refusals.

Layer 2 of each net (128 -> 128, lz_policy.hip mlp_i8_tail) runs on
v_mfma_i32_32x32x32_i8: B = layer 1's tanh outputs at scale 2^28 as they sit in the
accumulator (k-block kb = layer-1 tile kb; byte j of lane (env, h) = unit 32 kb +
row(j, h)), A = the weight digits (byte j of lane (m, h) = digit of W2[32 T + m][32 kb +
row(j, h)]); levels 6..3 in int32, y = ldexp(fma(float(L6 256 + L5), 2^16, float(L4 256 +
L3)), 24 - q_row - 28) + b2.
"""
import numpy as np
import pytest
import torch

from test_policy_f32_host import _random_policy, _row

F32 = np.float32
W2, HB = 4 * 64 * 16, 4 * 64 * 16 + 4 * 16 * 64 * 16 + 512 + 512 + 2048  # kF32W2 / kF32HB
SH2 = HB + 64                                                               # kF32Sh2
NET = SH2 + 256                                                             # kF32Net


@pytest.fixture(scope="module")
def pol():
    from gym_lorenz import policy

    return policy


def _f64_forward(sd, x):
    t = {k: np.asarray(v.numpy() if hasattr(v, "numpy") else v, np.float64) for k, v in sd.items()}
    X = x.astype(np.float64)
    out = []
    for net, hw, hb in (("policy_net", "action_net.weight", "action_net.bias"),
                        ("value_net", "value_net.weight", "value_net.bias")):
        h = np.tanh(X @ t["mlp_extractor.%s.0.weight" % net].T + t["mlp_extractor.%s.0.bias" % net])
        h = np.tanh(h @ t["mlp_extractor.%s.2.weight" % net].T + t["mlp_extractor.%s.2.bias" % net])
        out.append(h @ t[hw].T + t[hb])
    return out[0], out[1][:, 0]


@pytest.mark.parametrize("hidden", [128, 64])
def test_packed_digits_where_the_kernel_reads_them(pol, orc, hidden):
    _, sd = _random_policy(pol, 6, 2, seed=7, hidden=hidden)
    blob = pol.pack_policy_i8x4(sd, 6, 2)
    b32 = pol.pack_policy_f32(sd, 6, 2)
    same = np.ones(blob.size, bool)
    for base, key in ((0, "mlp_extractor.policy_net.2.weight"), (NET, "mlp_extractor.value_net.2.weight")):
        w = np.zeros((128, 128), F32)
        w[:hidden, :hidden] = sd[key].numpy()
        ops = np.frombuffer(blob[base + W2: base + W2 + 4 * 4 * 4 * 64 * 16].tobytes(),
                            np.int8).reshape(4, 4, 4, 64, 16)  # [T][kb][digit][lane][byte]
        sh = np.frombuffer(blob[base + SH2: base + SH2 + 256].tobytes(), np.int16).reshape(4, 2, 16)
        for T in range(4):
            for m in range(32):
                u = 32 * T + m
                q = orc.i8x_row_q(w[u])
                d = orc.i8x_digits(w[u], q)  # [128][4]
                for h in range(2):
                    ks = np.array([_row(j, h) for j in range(16)])
                    for kb in range(4):
                        for i in range(4):
                            assert np.array_equal(ops[T, kb, i, m + 32 * h], d[32 * kb + ks, i]), (u, h, kb, i)
            for h in range(2):
                for g in range(16):
                    assert sh[T, h, g] == 24 - orc.i8x_row_q(w[32 * T + _row(g, h)]) - 28
        same[base + W2: base + W2 + 4 * 16 * 64 * 16] = False
        same[base + SH2: base + NET] = False
    same[SH2 - 16: SH2] = False  # the format tag (kF32Tag = kF32HB + 48, in net 0)
    # everything else is the float32 blob
    assert np.array_equal(blob[same], b32[same])


def _level_forward(orc, sd, x):
    """orc_mlp_i8x4 restated in NumPy int64 / float64 (layer 2 only; layer 1 and the
    heads from the float32 oracle's own building blocks)"""
    t = {k: v.numpy() for k, v in sd.items()}
    outs = []
    for net, hw, hb in (("policy_net", "action_net.weight", "action_net.bias"),
                        ("value_net", "value_net.weight", "value_net.bias")):
        w1, b1 = t["mlp_extractor.%s.0.weight" % net], t["mlp_extractor.%s.0.bias" % net]
        w2, b2 = t["mlp_extractor.%s.2.weight" % net], t["mlp_extractor.%s.2.bias" % net]
        a1 = np.zeros((x.shape[0], 128), F32)
        for u in range(128):  # fmaf chain in k = 0, 1, ... (layer 1: k = 2s + h)
            acc = np.full(x.shape[0], b1[u], F32)
            for k in range(x.shape[1]):
                acc = (np.float64(w1[u, k]) * x[:, k].astype(np.float64) + acc).astype(F32)
            a1[:, u] = orc.tanh_tab(acc)
        ad = np.stack([orc.i8x_digits(a1[i], 28) for i in range(x.shape[0])]).astype(np.int64)
        a2 = np.zeros_like(a1)
        for u in range(128):
            q = orc.i8x_row_q(w2[u])
            wd = orc.i8x_digits(w2[u], q).astype(np.int64)
            L = np.zeros((x.shape[0], 7), np.int64)
            for i in range(4):
                for j in range(4):
                    if i + j >= 3:
                        L[:, i + j] += ad[:, :, j] @ wd[:, i]
            hi, lo = L[:, 6] * 256 + L[:, 5], L[:, 4] * 256 + L[:, 3]
            assert np.abs(hi).max() < 2 ** 24 and np.abs(lo).max() < 2 ** 31
            y = (np.float64(hi.astype(F32)) * 65536.0 + np.float64(lo.astype(F32))).astype(F32)
            a2[:, u] = orc.tanh_tab((np.ldexp(y, 24 - q - 28).astype(F32) + b2[u]).astype(F32))
        W, B = t[hw], t[hb]
        o = np.zeros((x.shape[0], W.shape[0]), F32)
        for r in range(W.shape[0]):
            part = []
            for h in range(2):
                acc = np.zeros(x.shape[0], F32)
                for T in range(4):
                    for g in range(16):
                        k = 32 * T + _row(g, h)
                        acc = (np.float64(W[r, k]) * a2[:, k].astype(np.float64) + acc).astype(F32)
                part.append(acc)
            o[:, r] = (part[0] + part[1]) + B[r]
        outs.append(o)
    return outs[0], outs[1][:, 0]


def test_oracle_equals_numpy_restatement(pol, orc):
    """orc_mlp_i8x4 == the same arithmetic in NumPy (obs_dim 2: layer 1's chain order is
    then the kernel's k = 2s + h without padding)."""
    _, sd = _random_policy(pol, 2, 1, seed=3)
    x = np.random.default_rng(3).normal(0, 2, (64, 2)).astype(F32)
    m, v = orc.mlp_f32(sd, x, precision="i8x4")
    me, ve = _level_forward(orc, sd, x)
    assert np.array_equal(m.view(np.uint32), me.view(np.uint32))
    assert np.array_equal(v.view(np.uint32), ve.view(np.uint32))


@pytest.mark.parametrize("sb3_init,scale", [(True, None), (False, 0.4), (False, 1.5)])
def test_accuracy_vs_float64(pol, orc, sb3_init, scale):
    """The i8x4 forward is as close to the float64 forward as the float32 one is."""
    if sb3_init:
        sd = {k: v.detach().clone() for k, v in pol.ActorCriticMlp(6, 2, seed=3).state_dict().items()}
    else:
        _, sd = _random_policy(pol, 6, 2, seed=11, scale=scale)
    x = np.random.default_rng(5).normal(0, 2.0, size=(4096, 6)).astype(F32)
    m8, v8 = orc.mlp_f32(sd, x, precision="i8x4")
    m32, v32 = orc.mlp_f32(sd, x)
    m64, v64 = _f64_forward(sd, x)
    e8 = max(np.abs(m8 - m64).max() / np.abs(m64).max(), np.abs(v8 - v64).max() / np.abs(v64).max())
    e32 = max(np.abs(m32 - m64).max() / np.abs(m64).max(), np.abs(v32 - v64).max() / np.abs(v64).max())
    print("vs float64: i8x4 %.2e, float32 %.2e" % (e8, e32))
    assert e8 <= 1.5 * e32 + 1e-7


def test_trained_pmsm_policies_teacher_forced(orc):
    """The reference's eight trained A2C policies (tests/golden/pmsm_closed_loop.npz) on
    the reference run's own observations: i8x4 actions within the float32 bar of
    test_f2_teacher_forced_vs_reference (5e-6)."""
    from test_policy_f32_host import GOLD, _sd, normalize_obs

    gold = np.load(GOLD)
    worst = 0.0
    for j in range(8):
        sd = _sd(gold, j, orc)
        m, _ = orc.mlp_f32(sd, normalize_obs(gold, j, gold["cpu_raw_obs"][j]), precision="i8x4")
        worst = max(worst, float(np.abs(np.clip(m, -1, 1) - gold["cpu_actions"][j]).max()))
    print("i8x4 vs the reference run's actions: max %.2e" % worst)
    assert worst <= 5e-6


def test_nan_obs_poisons_its_env_only(pol, orc):
    _, sd = _random_policy(pol, 6, 2, seed=2)
    x = np.random.default_rng(1).standard_normal((8, 6)).astype(F32)
    x[3, 1] = np.nan
    m, v = orc.mlp_f32(sd, x, precision="i8x4")
    assert np.isnan(m[3]).all() and np.isnan(v[3])
    keep = np.arange(8) != 3
    assert np.isfinite(m[keep]).all() and np.isfinite(v[keep]).all()


def test_pack_refuses_nonfinite_layer2(pol):
    from gym_lorenz import _native as nat

    _, sd = _random_policy(pol, 6, 2, seed=1)
    sd["mlp_extractor.value_net.2.weight"][5, 9] = float("nan")
    with pytest.raises(nat.LorenzEnvError):
        pol.pack_policy_i8x4(sd, 6, 2)
    pol.pack_policy_f32(sd, 6, 2)  # the float32 blob takes any float


@pytest.mark.parametrize("sb3_init", [True, False])
def test_i8x4_vs_torch_fp32_forward(pol, orc, sb3_init):
    """VERDICT r04 #4's torch bar for the MLP: the i8x4 forward's distance to SB3's own
    torch float32 forward is that of the float32 kernel's (measured 5.1e-7 / 3.6e-7 of the
    output scale, SB3 init, x ~ N(0, 2); the float32 oracle: 5.1e-7 / 2.9e-7 -- torch's
    own summation order is half of it)."""
    from test_policy_f32_host import _torch_forward

    if sb3_init:
        sd = {k: v.detach().clone() for k, v in pol.ActorCriticMlp(6, 2, seed=3).state_dict().items()}
    else:
        _, sd = _random_policy(pol, 6, 2, seed=4)
    x = np.random.default_rng(5).normal(0, 2.0, size=(4096, 6)).astype(F32)
    tm, tv = _torch_forward(sd, x)
    err = {}
    for prec in ("fp32", "i8x4"):
        m, v = orc.mlp_f32(sd, x, precision=prec)
        err[prec] = (np.abs(m - tm).max() / np.abs(tm).max(), np.abs(v - tv).max() / np.abs(tv).max())
    print("vs torch fp32: fp32 %.2e / %.2e, i8x4 %.2e / %.2e" % (err["fp32"] + err["i8x4"]))
    for j in range(2):
        assert err["i8x4"][j] <= 1.5 * err["fp32"][j] + 1e-7
        assert err["i8x4"][j] < 1e-6
