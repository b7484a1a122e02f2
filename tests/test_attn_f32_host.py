"""The float32 attention actor-critics on the host (no GPU): the oracle restatement and
the packed blob.

  * oracle.attn_f32 (lz_oracle.c orc_attn_f32, the kernel's operation order) against
    the plain torch float32 modules -- nn.MultiheadAttention / nn.LayerNorm as
    code/train.py:52-112 and code/lorenz_filter/train.py:54-132 build them: within
    ~1e-6 of the output scale (a different summation order and exp);
  * lz_attn_policy_pack_f32 / lz_attn_ln_policy_pack_f32: an emulation of the kernel's
    v_mfma_f32_16x16x4_f32 dataflow over the packed blob (lane (r, G) holds A[row r]
    [k = G] of every k-step; the accumulator of a 16-unit tile is the next k order) in
    float64 equals the oracle to rounding -- a wrong index map would be O(1) off;
  * the softmax exp (orc_exp_f32): <= 3 ulp over (-86, 0].
"""
import numpy as np
import pytest
import torch

F32 = np.float32


@pytest.fixture(scope="module")
def pol():
    from gym_lorenz import policy

    return policy


def _net(pol, in_dim, ln, seed):
    net = pol.ActorCriticAttn(in_dim, 2, seed=seed, layer_norm=ln)
    g = torch.Generator().manual_seed(seed + 7)
    with torch.no_grad():
        for p in net.parameters():
            p.add_(torch.randn(p.shape, generator=g) * 0.05)
    return net


@pytest.mark.parametrize("ln,in_dim", [(False, 6), (True, 24), (True, 6)])
def test_oracle_attn_f32_vs_torch_fp32(pol, orc, ln, in_dim):
    net = _net(pol, in_dim, ln, seed=3)
    x = torch.randn(3000, in_dim, generator=torch.Generator().manual_seed(1)) * 2.0
    m, v = orc.attn_f32(net.state_dict(), x.numpy())
    with torch.no_grad():
        mt, vt = net(x)
    dm = np.abs(m - mt.numpy()).max() / max(1.0, np.abs(mt.numpy()).max())
    dv = np.abs(v - vt.numpy()).max() / max(1.0, np.abs(vt.numpy()).max())
    print("attention f32 oracle vs torch fp32 (ln=%s): mean %.2e, value %.2e" % (ln, dm, dv))
    assert dm < 2e-6 and dv < 2e-6


def test_exp_f32_accuracy(orc):
    xs = np.concatenate([np.linspace(-86, 0, 2001), -np.logspace(-8, 0, 300)]).astype(F32)
    e = orc.exp_f32(xs).astype(np.float64)
    t = np.exp(xs.astype(np.float64))
    assert (np.abs(e - t) / np.spacing(t.astype(F32))).max() <= 3.0
    assert np.isnan(orc.exp_f32(np.array([np.nan], F32))[0])
    assert orc.exp_f32(np.array([-np.inf, -90.0], F32)).tolist() == [0.0, 0.0]


# ------------------------------------------------------- emulation of the blob dataflow
# byte offsets, gym-lorenz_amd/csrc/lz_internal.h kAF*
FC1W, FC1B = 0, 16384
KW, VW, QW, OW = 16896, 17920, 18944, 19968
KB, VB, QB, OB, GAM, BET = 20992, 21056, 21120, 21184, 21248, 21312
POSTW, POSTB, EXT = 21376, 54144, 54400
N1, N2, NB1, NB2, NH, NHB, NET = 0, 32768, 98304, 98816, 99328, 101376, 102400
PI, VF = EXT, EXT + NET


def _tile(a_op, inputs):
    """One 16-row tile of v_mfma_f32_16x16x4_f32 chains: a_op [ksteps][64 lanes] (lane
    16G + r: A[row r][k = G]), inputs(s, G) -> [n] B values.  Returns [n, 16]."""
    out = 0.0
    for s in range(a_op.shape[0]):
        for G in range(4):
            out = out + a_op[s, 16 * G:16 * G + 16][None, :] * inputs(s, G)[:, None]
    return out


def _tile_in(acc):
    """A [n, 16] accumulator as the next k order: k-step s, group G -> unit 4G + s."""
    return lambda s, G: acc[:, 4 * G + s]


def _emulate(blob, x, ln, A):
    f = blob.view(F32).astype(np.float64)

    def fl(off, cnt):
        return f[off // 4: off // 4 + cnt]

    n, I = x.shape
    xd = x.astype(np.float64)
    fc1 = fl(FC1W, 8 * 2 * 64 * 4).reshape(8, 2, 64, 4).transpose(0, 1, 3, 2).reshape(8, 8, 64)
    tok = []
    for t in range(8):
        acc = fl(FC1B, 128)[16 * t:16 * t + 16][None, :] + _tile(
            fc1[t], lambda s, G: xd[:, 4 * s + G] if 4 * s + G < I else np.zeros(n))
        tok.append(np.maximum(acc, 0.0))

    def w4(off):
        return fl(off, 256).reshape(64, 4).T  # [4 k-steps][64 lanes]

    K = [fl(KB, 16)[None] + _tile(w4(KW), _tile_in(tk)) for tk in tok]
    V = [fl(VB, 16)[None] + _tile(w4(VW), _tile_in(tk)) for tk in tok]
    post = np.repeat(fl(POSTB, 64)[None], n, 0)
    pw = fl(POSTW, 4 * 8 * 64 * 4).reshape(4, 8, 64, 4)
    for i in range(8):
        q = fl(QB, 16)[None] + _tile(w4(QW), _tile_in(tok[i]))
        att = np.zeros((n, 16))
        for hd in range(4):
            sl = slice(4 * hd, 4 * hd + 4)
            sc = np.stack([(q[:, sl] * K[j][:, sl]).sum(1) for j in range(8)], 1)
            e = np.exp(sc - sc.max(1, keepdims=True))
            w = e / e.sum(1, keepdims=True)
            att[:, sl] = sum(w[:, j:j + 1] * V[j][:, sl] for j in range(8))
        y = fl(OB, 16)[None] + _tile(w4(OW), _tile_in(att))
        if ln:
            z = y + tok[i]
            z = (z - z.mean(1, keepdims=True)) / np.sqrt(z.var(1, keepdims=True) + 1e-5)
            y = z * fl(GAM, 16)[None] + fl(BET, 16)[None]
        for u in range(4):
            post[:, 16 * u:16 * u + 16] += _tile(pw[u, i].T, _tile_in(y))
    feat = np.maximum(post, 0.0)

    def net(base, rows):
        g = lambda off, cnt: fl(base + off, cnt)  # noqa: E731
        w1 = g(N1, 8 * 4 * 64 * 4).reshape(8, 4, 64, 4).transpose(0, 1, 3, 2).reshape(8, 16, 64)
        w2 = g(N2, 8 * 8 * 64 * 4).reshape(8, 8, 64, 4).transpose(0, 1, 3, 2).reshape(8, 32, 64)
        a1 = np.concatenate([np.tanh(g(NB1, 128)[16 * t:16 * t + 16][None] + _tile(
            w1[t], lambda s, G: feat[:, 16 * (s // 4) + 4 * G + s % 4])) for t in range(8)], 1)
        a2 = np.concatenate([np.tanh(g(NB2, 128)[16 * t:16 * t + 16][None] + _tile(
            w2[t], lambda s, G: a1[:, 16 * (s // 4) + 4 * G + s % 4])) for t in range(8)], 1)
        hw = g(NH, 4 * 128).reshape(4, 128)[:rows]
        return a2 @ hw.T + g(NHB, 4)[:rows][None]

    return net(PI, A), net(VF, 1)[:, 0]


@pytest.mark.parametrize("ln,in_dim", [(False, 6), (True, 24)])
def test_attn_f32_blob_dataflow_equals_oracle(pol, orc, ln, in_dim):
    net = _net(pol, in_dim, ln, seed=5)
    sd = net.state_dict()
    blob = (pol.pack_attn_ln_policy_f32 if ln else pol.pack_attn_policy_f32)(sd, in_dim, 2)
    from gym_lorenz import _native as nat

    assert blob.size == nat.lib.lz_attn_policy_f32_blob_bytes()
    x = (np.random.default_rng(2).normal(0, 2, (400, in_dim))).astype(F32)
    me, ve = _emulate(blob, x, ln, 2)
    mo, vo = orc.attn_f32(sd, x)
    assert np.abs(me - mo).max() < 2e-5 * max(1.0, np.abs(mo).max())
    assert np.abs(ve - vo).max() < 2e-5 * max(1.0, np.abs(vo).max())


def test_attn_f32_pack_rejects_bad_shapes(pol):
    net = _net(pol, 6, False, seed=1)
    sd = dict(net.state_dict())
    with pytest.raises(ValueError):
        pol.pack_attn_policy_f32(sd, 5, 2)  # wrong obs width
    from gym_lorenz import _native as nat

    with pytest.raises(nat.LorenzEnvError):
        pol.pack_attn_policy_f32(_net(pol, 9, False, seed=1).state_dict(), 9, 2)  # obs_dim > 8


# ------------------------------------------------------- pinned to the reference's classes
def _attn_ref(tag):
    from conftest import golden

    g = golden("attn_ref")
    pre = tag + "/"
    sd = {k[len(pre):]: torch.from_numpy(v) for k, v in g.items()
          if k.startswith(pre) and k[len(pre):] not in ("x", "features", "mean", "value")}
    return sd, g[pre + "x"], g[pre + "features"], g[pre + "mean"], g[pre + "value"]


@pytest.mark.parametrize("tag", ["plain", "ln"])
def test_oracle_attn_f32_vs_reference_classes(orc, pol, tag):
    """tests/golden/attn_ref.npz was produced by the reference's own
    AttentionFeaturesExtractor classes (code/train.py:52-94; code/lorenz_filter/train.py:
    55-103, residual + LayerNorm, on 24-dim VecFrameStack(4) inputs) inside SB3's policy
    layout, in torch float32 (tests/golden/make_attn_ref.py).  The oracle the float32
    kernels are bit-exact against (orc_attn_f32) reproduces the features, action means
    and values within 2e-6 of the output scale; so does this package's torch
    restatement (gym_lorenz.policy.ActorCriticAttn, loaded with the same state_dict)."""
    sd, x, f_ref, m_ref, v_ref = _attn_ref(tag)
    m, v, f = orc.attn_f32(sd, x, return_features=True)

    def rel(a, b):
        return float(np.abs(a - b).max() / max(1.0, np.abs(b).max()))

    df, dm, dv = rel(f, f_ref), rel(m, m_ref), rel(v, v_ref)
    print("orc_attn_f32 vs the reference's %s extractor: features %.2e, mean %.2e, value %.2e"
          % (tag, df, dm, dv))
    assert df < 2e-6 and dm < 2e-6 and dv < 2e-6
    # the softmax is far from uniform on these weights (the fixture exercises attention)
    net = pol.ActorCriticAttn(x.shape[1], 2, layer_norm=tag == "ln")
    net.load_state_dict(sd)
    with torch.no_grad():
        mt, vt = net(torch.from_numpy(x))
        xs = torch.relu(net.features_extractor.fc1(torch.from_numpy(x[:64]))).view(-1, 8, 16)
        _, w = net.features_extractor.attention_layer(xs, xs, xs)
    assert rel(mt.numpy(), m_ref) < 2e-6 and rel(vt.numpy(), v_ref) < 2e-6
    assert float(w.max()) > 0.5  # some query attends mostly to one token
