"""Host side of the fused policy rollout, no GPU needed.

- lz_policy_pack lays the SB3 actor-critic out as the MFMA fragments the kernel
  reads: checked by emulating v_mfma_f32_32x32x16_bf16 on the CPU with the operand /
  result layouts of the CDNA4 guide (A: lane (r, h) holds A[r][8h + j]; B: lane (r, h)
  holds B[8h + j][r]; D: lane (c, h) register g holds D[(g&3) + 8(g>>2) + 4h][c]) and
  running the kernel's exact dataflow (accumulator -> tanh -> bf16 -> next B operand)
  over the packed blob; the result must equal the torch bf16 restatement
  (policy.reference_forward_bf16) up to fp32 summation order.
- the SB3 GAE restatement (oracle/sb3_buffer.py) against a hand-derived case.
- the public structs' layout against the ctypes mirror.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest
import torch

from conftest import ROOT


@pytest.fixture(scope="module")
def pol():
    from gym_lorenz import policy

    return policy


def _bf16(x):
    return torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(torch.bfloat16).to(
        torch.float32).numpy()


def _unpack(blob, off, count):
    u = blob[off: off + count * 64 * 16].view(np.uint16).astype(np.uint32) << 16
    return u.view(np.float32).reshape(count, 64, 8)


def _mfma(a, b, c):
    """v_mfma_f32_32x32x16_bf16 on fragments a, b [64, 8] and accumulator c [64, 16]."""
    A = np.zeros((32, 16), np.float64)
    B = np.zeros((16, 32), np.float64)
    for lane in range(64):
        r, h = lane & 31, lane >> 5
        A[r, 8 * h: 8 * h + 8] = a[lane]
        B[8 * h: 8 * h + 8, r] = b[lane]
    D = A @ B
    out = c.astype(np.float64).copy()
    for lane in range(64):
        col, h = lane & 31, lane >> 5
        for g in range(16):
            out[lane, g] += D[(g & 3) + 8 * (g >> 2) + 4 * h, col]
    return out.astype(np.float32)


def _act(c):
    """tanh of the pre-scaled accumulator (the packer folds s = 2/ln 2 into the tanh
    layers), then registers 8s..8s+7 -> bf16 B fragment of k-step s."""
    t = _bf16(np.tanh(c.astype(np.float64) / np.float64(np.float32(2.8853900817779268)))
              .astype(np.float32))
    return [t[:, 0:8], t[:, 8:16]]


def _emulate(pol, blob, obs):
    """The kernel's forward on one 32-env tile; returns (mean [32, A], value [32])."""
    from gym_lorenz import _native  # noqa: F401  (library must load)

    O = obs.shape[1]
    L = {k: v for k, v in (
        ("W1", 0), ("W2", 4 * 64 * 16), ("W3", 4 * 64 * 16 + 4 * 8 * 64 * 16))}
    L["B1"] = L["W3"] + 8 * 64 * 16
    L["B2"] = L["B1"] + 512
    L["B3"] = L["B2"] + 512
    net_bytes = L["B3"] + 128
    x = np.zeros((64, 8), np.float32)
    x[:32, :O] = _bf16(obs)
    outs = []
    for net in (0, net_bytes):
        w1 = _unpack(blob, net + L["W1"], 4)
        w2 = _unpack(blob, net + L["W2"], 32)
        w3 = _unpack(blob, net + L["W3"], 8)
        b1 = blob[net + L["B1"]: net + L["B1"] + 512].view(np.float32).reshape(4, 2, 16)
        b2 = blob[net + L["B2"]: net + L["B2"] + 512].view(np.float32).reshape(4, 2, 16)
        b3 = blob[net + L["B3"]: net + L["B3"] + 128].view(np.float32).reshape(2, 16)
        lane_h = np.arange(64) >> 5
        h1 = []
        for t in range(4):
            h1 += _act(_mfma(w1[t], x, b1[t][lane_h]))
        h2 = []
        for t in range(4):
            c = b2[t][lane_h]
            for kk in range(8):
                c = _mfma(w2[t * 8 + kk], h1[kk], c)
            h2 += _act(c)
        c = b3[lane_h]
        for kk in range(8):
            c = _mfma(w3[kk], h2[kk], c)
        outs.append(c)
    # head row j < 4 sits in lane half 0, register j
    return outs[0][:32, :4], outs[1][:32, 0]


def _random_policy(pol, O, A, seed):
    net = pol.ActorCriticMlp(O, A, seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():  # non-degenerate weights: ortho init's 0.01 head gain hides errors
        for p in net.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * (0.4 if p.dim() > 1 else 0.3))
    return {k: v.detach().clone() for k, v in net.state_dict().items()}


@pytest.mark.parametrize("O,A", [(6, 2), (6, 3), (8, 3)])
def test_pack_layout_matches_mfma_dataflow(pol, O, A):
    sd = _random_policy(pol, O, A, seed=O * 10 + A)
    blob = pol.pack_policy(sd, O, A)
    obs = np.random.default_rng(O + A).normal(0, 1.5, size=(32, O)).astype(np.float32)
    mean, value = _emulate(pol, blob, obs)
    ref_mean, ref_value = pol.reference_forward_bf16(sd, obs)
    np.testing.assert_allclose(mean[:, :A], ref_mean.numpy(), rtol=0, atol=2e-4)
    np.testing.assert_allclose(value, ref_value.numpy(), rtol=0, atol=2e-4)
    # padded head rows are exact zeros
    assert np.all(mean[:, A:] == 0)


def test_pack_rejects_bad_shapes(pol):
    sd = _random_policy(pol, 6, 2, seed=0)
    with pytest.raises(ValueError):
        pol.pack_policy(sd, 6, 3)
    bad = dict(sd)
    del bad["log_std"]
    with pytest.raises(KeyError):
        pol.pack_policy(bad, 6, 2)
    from gym_lorenz import _native as nat
    with pytest.raises(nat.LorenzEnvError):
        big = _random_policy(pol, 9, 2, seed=1)
        pol.pack_policy(big, 9, 2)


def test_sb3_gae_restatement_hand_case():
    from oracle.sb3_buffer import compute_returns_and_advantage

    rew = np.array([[1.0], [2.0]], np.float32)
    val = np.array([[0.5], [0.25]], np.float32)
    starts = np.array([[1.0], [0.0]], np.float32)
    adv, ret = compute_returns_and_advantage(rew, val, starts, np.array([4.0], np.float32),
                                             np.array([False]), 0.5, 0.5)
    d1 = 2.0 + 0.5 * 4.0 - 0.25
    d0 = 1.0 + 0.5 * 0.25 - 0.5
    assert adv[1, 0] == np.float32(d1)
    assert adv[0, 0] == np.float32(d0 + 0.25 * d1)
    assert ret[0, 0] == adv[0, 0] + val[0, 0]
    adv2, _ = compute_returns_and_advantage(rew, val, np.array([[1.0], [1.0]], np.float32),
                                            np.array([4.0], np.float32), np.array([True]), 0.5,
                                            0.5)
    assert adv2[1, 0] == np.float32(2.0 - 0.25) and adv2[0, 0] == np.float32(1.0 - 0.5)


def test_policy_structs_match_header(tmp_path):
    from gym_lorenz import _native as nat

    c = tmp_path / "probe.c"
    c.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "lorenz_env.h"\n'
        "int main(void){printf(\"%zu %zu %zu %zu %zu %zu %zu\\n\", sizeof(lz_mlp_policy),"
        " offsetof(lz_mlp_policy, log_std), sizeof(lz_policy_rollout_args),"
        " offsetof(lz_policy_rollout_args, norm_eps), offsetof(lz_policy_rollout_args, act_low),"
        " offsetof(lz_policy_rollout_args, cap), offsetof(lz_policy_rollout_args, n_done));"
        "return 0;}\n")
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)])
    got = [int(v) for v in subprocess.check_output([str(exe)]).split()]
    P, R = nat.LzMlpPolicy, nat.LzPolicyRolloutArgs
    want = [ctypes.sizeof(P), P.log_std.offset, ctypes.sizeof(R), R.norm_eps.offset,
            R.act_low.offset, R.cap.offset, R.n_done.offset]
    assert got == want
    assert nat.lib.lz_policy_blob_bytes() == 92480


def test_attn_policy_struct_matches_header(tmp_path):
    from gym_lorenz import _native as nat

    c = tmp_path / "probe.c"
    c.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "lorenz_env.h"\n'
        'int main(void){printf("%zu %zu %zu %zu %zu\\n", sizeof(lz_attn_policy),'
        " offsetof(lz_attn_policy, post_b), offsetof(lz_attn_policy, log_std),"
        " sizeof(lz_attn_ln_policy), offsetof(lz_attn_ln_policy, ln_b));return 0;}\n")
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)])
    got = [int(v) for v in subprocess.check_output([str(exe)]).split()]
    P = nat.LzAttnPolicy
    Q = nat.LzAttnLnPolicy
    assert got == [ctypes.sizeof(P), P.post_b.offset, P.log_std.offset, ctypes.sizeof(Q),
                   Q.ln_b.offset]
    assert nat.lib.lz_attn_policy_blob_bytes() == 140608
    assert nat.lib.lz_attn_ln_policy_blob_bytes() == 145984


def test_sb3_framestack_restatement_hand_case():
    from oracle.sb3_framestack import StackedObservations

    so = StackedObservations(2, 3, 2)
    st = so.reset(np.array([[1, 2], [3, 4]], np.float32))
    assert st.tolist() == [[0, 0, 0, 0, 1, 2], [0, 0, 0, 0, 3, 4]]
    infos = [{}, {"terminal_observation": np.array([9, 9], np.float32)}]
    st, infos = so.update(np.array([[5, 6], [7, 8]], np.float32), np.array([False, True]), infos)
    assert st.tolist() == [[0, 0, 1, 2, 5, 6], [0, 0, 0, 0, 7, 8]]
    assert infos[1]["terminal_observation"].tolist() == [0, 0, 3, 4, 9, 9]


# ---------------------------------------------------------------- attention extractor
# lz_internal.h kAtt* layout (bytes)
def _attn_layout():
    L = {"Fc1W": 0}
    L["Fc1B"] = L["Fc1W"] + 4 * 64 * 16
    L["KvW"] = L["Fc1B"] + 4 * 2 * 16 * 4
    L["KvB"] = L["KvW"] + 64 * 16
    L["QW"] = L["KvB"] + 2 * 16 * 4
    L["QB"] = L["QW"] + 64 * 16
    L["PostW"] = L["QB"] + 2 * 16 * 4
    L["PostB"] = L["PostW"] + 8 * 2 * 64 * 16
    L["Ext"] = L["PostB"] + 2 * 2 * 16 * 4
    N = {"W1": 0}
    N["W2"] = N["W1"] + 4 * 4 * 64 * 16
    N["W3"] = N["W2"] + 4 * 8 * 64 * 16
    N["B1"] = N["W3"] + 8 * 64 * 16
    N["B2"] = N["B1"] + 512
    N["B3"] = N["B2"] + 512
    N["Net"] = N["B3"] + 128
    return L, N


def _relu_frag(c):
    t = _bf16(np.where(c < 0, np.float32(0), c))  # torch.relu keeps NaN
    return [t[:, 0:8], t[:, 8:16]]


def _emulate_attn(blob, obs):
    """lz_rollout_policy_attn's forward on one 32-env tile over the packed blob."""
    L, N = _attn_layout()
    f32 = lambda off, n: blob[off: off + 4 * n].view(np.float32)  # noqa: E731
    lane_h = np.arange(64) >> 5
    O = obs.shape[1]
    x = np.zeros((64, 8), np.float32)
    x[:32, :O] = _bf16(obs)
    fc1 = _unpack(blob, L["Fc1W"], 4)
    b1 = f32(L["Fc1B"], 128).reshape(4, 2, 16)
    tok = []
    for t in range(4):
        tok += _relu_frag(_mfma(fc1[t], x, b1[t][lane_h]))
    wkv = _unpack(blob, L["KvW"], 1)[0]
    bkv = f32(L["KvB"], 32).reshape(2, 16)[lane_h]
    kv = np.stack([_mfma(wkv, tok[t], bkv) for t in range(8)], 1)  # [64, token, 16]
    wq = _unpack(blob, L["QW"], 1)[0]
    bq = f32(L["QB"], 32).reshape(2, 16)[lane_h]
    wp = _unpack(blob, L["PostW"], 16)
    bp = f32(L["PostB"], 64).reshape(2, 2, 16)
    f0, f1 = bp[0][lane_h], bp[1][lane_h]
    for i in range(8):
        q = _mfma(wq, tok[i], bq)
        o = np.zeros((64, 8), np.float32)
        for hh in range(2):
            s = np.einsum("ld,ljd->lj", q[:, 4 * hh: 4 * hh + 4], kv[:, :, 4 * hh: 4 * hh + 4])
            p = np.exp2(s - s.max(1, keepdims=True))
            o[:, 4 * hh: 4 * hh + 4] = np.einsum("lj,ljd->ld", p, kv[:, :, 8 + 4 * hh: 12 + 4 * hh]) * (
                np.float32(1) / p.sum(1, keepdims=True))
        a = _bf16(o)
        f0 = _mfma(wp[2 * i], a, f0)
        f1 = _mfma(wp[2 * i + 1], a, f1)
    feat = _relu_frag(f0) + _relu_frag(f1)
    outs = []
    for net in (L["Ext"], L["Ext"] + N["Net"]):
        w1 = _unpack(blob, net + N["W1"], 16)
        w2 = _unpack(blob, net + N["W2"], 32)
        w3 = _unpack(blob, net + N["W3"], 8)
        nb1 = f32(net + N["B1"], 128).reshape(4, 2, 16)
        nb2 = f32(net + N["B2"], 128).reshape(4, 2, 16)
        nb3 = f32(net + N["B3"], 32).reshape(2, 16)
        h1 = []
        for t in range(4):
            c = nb1[t][lane_h]
            for s in range(4):
                c = _mfma(w1[t * 4 + s], feat[s], c)
            h1 += _act(c)
        h2 = []
        for t in range(4):
            c = nb2[t][lane_h]
            for kk in range(8):
                c = _mfma(w2[t * 8 + kk], h1[kk], c)
            h2 += _act(c)
        c = nb3[lane_h]
        for kk in range(8):
            c = _mfma(w3[kk], h2[kk], c)
        outs.append(c)
    return outs[0][:32, :4], outs[1][:32, 0]


def _random_attn_policy(pol, O, A, seed, scale=0.4):
    net = pol.ActorCriticAttn(O, A, seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for p in net.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * (scale if p.dim() > 1 else 0.3))
    return net, {k: v.detach().clone() for k, v in net.state_dict().items()}


@pytest.mark.parametrize("O,A", [(6, 2), (3, 3), (8, 1)])
def test_attn_pack_layout_matches_mfma_dataflow(pol, O, A):
    _, sd = _random_attn_policy(pol, O, A, seed=O * 10 + A)
    blob = pol.pack_attn_policy(sd, O, A)
    assert blob.size == 140608
    obs = np.random.default_rng(O + A).normal(0, 1.5, size=(32, O)).astype(np.float32)
    mean, value = _emulate_attn(blob, obs)
    ref_mean, ref_value = pol.reference_forward_attn_bf16(sd, obs)
    # same bf16 roundings; fp32 summation order may flip a rounding boundary
    np.testing.assert_allclose(mean[:, :A], ref_mean.numpy(), rtol=0, atol=5e-3)
    np.testing.assert_allclose(value, ref_value.numpy(), rtol=0, atol=5e-3)
    assert np.median(np.abs(mean[:, :A] - ref_mean.numpy())) < 1e-4
    assert np.all(mean[:, A:] == 0)


@pytest.mark.parametrize("sb3_init", [False, True])
def test_attn_restatement_vs_fp32_module(pol, sb3_init):
    """The bf16 restatement (q pre-scale, base-2 softmax, out_proj folded into
    post_attention_fc) against the plain fp32 module of code/train.py:52-95 under
    nn.MultiheadAttention: agreement to bf16 accuracy."""
    if sb3_init:
        net = pol.ActorCriticAttn(6, 2, seed=3)
        net.log_std.data.zero_()
        sd = net.state_dict()
    else:
        net, sd = _random_attn_policy(pol, 6, 2, seed=7, scale=0.25)
    obs = np.random.default_rng(5).normal(0, 1.0, size=(512, 6)).astype(np.float32)
    with torch.no_grad():
        m32, v32 = net(torch.from_numpy(obs))
    mb, vb = pol.reference_forward_attn_bf16(sd, obs)
    for got, want in ((mb, m32), (vb, v32)):
        err = (got - want).abs()
        scale = want.abs().max().item()
        assert err.max().item() <= 0.03 * scale + 1e-4, (err.max().item(), scale)
        assert err.mean().item() <= 0.006 * scale + 1e-5


def test_attn_state_dict_keys_match_sb3(pol):
    """The module's state_dict keys are SB3's for code/train.py's policy (the shared
    extractor under features_extractor.); pi_features_extractor. aliases are accepted."""
    net = pol.ActorCriticAttn(6, 2, seed=0)
    sd = net.state_dict()
    for k in pol.ATTN_FE_KEYS:
        assert pol.FE + k in sd
    for k in pol.KEYS:
        assert k in sd
    assert pol.is_attention_policy(sd) and not pol.is_attention_policy(
        pol.ActorCriticMlp(6, 2, seed=0).state_dict())
    alias = {("pi_" + k if k.startswith(pol.FE) else k): v for k, v in sd.items()}
    assert np.array_equal(pol.pack_attn_policy(alias, 6, 2), pol.pack_attn_policy(sd, 6, 2))
    bad = dict(sd)
    del bad[pol.FE + "attention_layer.in_proj_bias"]
    with pytest.raises(KeyError):
        pol.pack_attn_policy(bad, 6, 2)
    with pytest.raises(ValueError):
        pol.pack_attn_policy(sd, 6, 3)


# ------------------------------------------- residual + LayerNorm variant (lorenz_filter)
def _ln_layout():
    L = {"Fc1W": 0}
    L["Fc1B"] = L["Fc1W"] + 4 * 2 * 64 * 16
    L["KvW"] = L["Fc1B"] + 512
    L["KvB"] = L["KvW"] + 1024
    L["QW"] = L["KvB"] + 128
    L["QB"] = L["QW"] + 1024
    L["OutW"] = L["QB"] + 128
    L["OutB"] = L["OutW"] + 1024
    L["Gamma"] = L["OutB"] + 128
    L["Beta"] = L["Gamma"] + 64
    L["PostW"] = L["Beta"] + 64
    L["PostB"] = L["PostW"] + 8 * 2 * 64 * 16
    L["Ext"] = L["PostB"] + 256
    return L


def _emulate_attn_ln(blob, x_in):
    """lz_rollout_policy_attn_stack's forward on one 32-env tile (x_in: [32, <=32] the
    stacked policy input) over the packed kLn blob."""
    L = _ln_layout()
    _, N = _attn_layout()
    f32 = lambda off, n: blob[off: off + 4 * n].view(np.float32)  # noqa: E731
    lane_h = np.arange(64) >> 5
    I = x_in.shape[1]
    xin = np.zeros((32, 32), np.float32)
    xin[:, :I] = _bf16(x_in)
    xs = []
    for s in range(2):  # k-step s: half h holds stacked dims 16s + 8h + j
        f = np.zeros((64, 8), np.float32)
        f[:32] = xin[:, 16 * s: 16 * s + 8]
        f[32:] = xin[:, 16 * s + 8: 16 * s + 16]
        xs.append(f)
    fc1 = _unpack(blob, L["Fc1W"], 8)
    b1 = f32(L["Fc1B"], 128).reshape(4, 2, 16)
    tok = []
    for t in range(4):
        c = b1[t][lane_h]
        for s in range(2):
            c = _mfma(fc1[t * 2 + s], xs[s], c)
        tok += _relu_frag(c)
    wkv = _unpack(blob, L["KvW"], 1)[0]
    kv = np.stack([_mfma(wkv, tok[t], f32(L["KvB"], 32).reshape(2, 16)[lane_h]) for t in range(8)], 1)
    wq = _unpack(blob, L["QW"], 1)[0]
    bq = f32(L["QB"], 32).reshape(2, 16)[lane_h]
    wo = _unpack(blob, L["OutW"], 1)[0]
    bo = f32(L["OutB"], 32).reshape(2, 16)[lane_h]
    gam = f32(L["Gamma"], 16).reshape(2, 8)[lane_h]
    bet = f32(L["Beta"], 16).reshape(2, 8)[lane_h]
    wp = _unpack(blob, L["PostW"], 16)
    bp = f32(L["PostB"], 64).reshape(2, 2, 16)
    f0, f1 = bp[0][lane_h], bp[1][lane_h]
    for i in range(8):
        q = _mfma(wq, tok[i], bq)
        o = np.zeros((64, 8), np.float32)
        for hh in range(2):
            s_ = np.einsum("ld,ljd->lj", q[:, 4 * hh: 4 * hh + 4], kv[:, :, 4 * hh: 4 * hh + 4])
            p = np.exp2(s_ - s_.max(1, keepdims=True))
            o[:, 4 * hh: 4 * hh + 4] = np.einsum("lj,ljd->ld", p, kv[:, :, 8 + 4 * hh: 12 + 4 * hh]) * (
                np.float32(1) / p.sum(1, keepdims=True))
        y = _mfma(wo, _bf16(o), bo)[:, :8]
        z = y + tok[i]
        tot = z.sum(1) + np.roll(z.sum(1), 32)  # the two halves' partial sums
        z = z - (tot * np.float32(0.0625))[:, None]
        sq = (z * z).sum(1)
        var = (sq + np.roll(sq, 32)) * np.float32(0.0625)
        u = _bf16(z / np.sqrt(var + np.float32(1e-5))[:, None] * gam + bet)
        f0 = _mfma(wp[2 * i], u, f0)
        f1 = _mfma(wp[2 * i + 1], u, f1)
    feat = _relu_frag(f0) + _relu_frag(f1)
    outs = []
    for net in (L["Ext"], L["Ext"] + N["Net"]):
        w1 = _unpack(blob, net + N["W1"], 16)
        w2 = _unpack(blob, net + N["W2"], 32)
        w3 = _unpack(blob, net + N["W3"], 8)
        nb1 = f32(net + N["B1"], 128).reshape(4, 2, 16)
        nb2 = f32(net + N["B2"], 128).reshape(4, 2, 16)
        nb3 = f32(net + N["B3"], 32).reshape(2, 16)
        h1 = []
        for t in range(4):
            c = nb1[t][lane_h]
            for s in range(4):
                c = _mfma(w1[t * 4 + s], feat[s], c)
            h1 += _act(c)
        h2 = []
        for t in range(4):
            c = nb2[t][lane_h]
            for kk in range(8):
                c = _mfma(w2[t * 8 + kk], h1[kk], c)
            h2 += _act(c)
        c = nb3[lane_h]
        for kk in range(8):
            c = _mfma(w3[kk], h2[kk], c)
        outs.append(c)
    return outs[0][:32, :4], outs[1][:32, 0]


def _random_attn_ln_policy(pol, I, A, seed, scale=0.3):
    net = pol.ActorCriticAttn(I, A, seed=seed, layer_norm=True)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for name, p in net.named_parameters():
            if "layer_norm" in name:  # gains around 1, offsets small
                p.copy_((1.0 if name.endswith("weight") else 0.0)
                        + 0.2 * torch.randn(p.shape, generator=g))
            else:
                p.copy_(torch.randn(p.shape, generator=g) * (scale if p.dim() > 1 else 0.3))
    return net, {k: v.detach().clone() for k, v in net.state_dict().items()}


@pytest.mark.parametrize("I,A", [(24, 2), (6, 2), (32, 3), (13, 1)])
def test_attn_ln_pack_layout_matches_mfma_dataflow(pol, I, A):
    _, sd = _random_attn_ln_policy(pol, I, A, seed=I + A)
    blob = pol.pack_attn_ln_policy(sd, I, A)
    assert blob.size == 145984
    x = np.random.default_rng(I).normal(0, 1.0, size=(32, I)).astype(np.float32)
    mean, value = _emulate_attn_ln(blob, x)
    ref_mean, ref_value = pol.reference_forward_attn_ln_bf16(sd, x)
    np.testing.assert_allclose(mean[:, :A], ref_mean.numpy(), rtol=0, atol=5e-3)
    np.testing.assert_allclose(value, ref_value.numpy(), rtol=0, atol=5e-3)
    assert np.median(np.abs(mean[:, :A] - ref_mean.numpy())) < 1e-4
    assert np.all(mean[:, A:] == 0)


@pytest.mark.parametrize("sb3_init", [False, True])
def test_attn_ln_restatement_vs_fp32_module(pol, sb3_init):
    """The bf16 restatement of code/lorenz_filter/train.py's extractor (residual on the
    bf16 tokens, fp32 LayerNorm) against the plain fp32 module: bf16 accuracy."""
    if sb3_init:
        net = pol.ActorCriticAttn(24, 2, seed=3, layer_norm=True)
        sd = net.state_dict()
    else:
        net, sd = _random_attn_ln_policy(pol, 24, 2, seed=9)
    x = np.random.default_rng(5).normal(0, 1.0, size=(512, 24)).astype(np.float32)
    with torch.no_grad():
        m32, v32 = net(torch.from_numpy(x))
    mb, vb = pol.reference_forward_attn_ln_bf16(sd, x)
    for got, want in ((mb, m32), (vb, v32)):
        err = (got - want).abs()
        scale = want.abs().max().item()
        assert err.max().item() <= 0.04 * scale + 1e-4, (err.max().item(), scale)
        assert err.mean().item() <= 0.008 * scale + 1e-5, (err.mean().item(), scale)


def test_attn_ln_keys_and_errors(pol):
    net = pol.ActorCriticAttn(24, 2, seed=0, layer_norm=True)
    sd = net.state_dict()
    assert pol.is_attention_ln_policy(sd) and pol.is_attention_policy(sd)
    assert not pol.is_attention_ln_policy(pol.ActorCriticAttn(6, 2, seed=0).state_dict())
    with pytest.raises(ValueError):
        pol.pack_attn_ln_policy(sd, 6, 2)  # fc1 is [128, 24]
    from gym_lorenz import _native as nat
    big = pol.ActorCriticAttn(40, 2, seed=0, layer_norm=True).state_dict()
    with pytest.raises(nat.LorenzEnvError):
        pol.pack_attn_ln_policy(big, 40, 2)


@pytest.mark.parametrize("H", [64, 32, 100])
def test_pack_narrow_nets_zero_padded(pol, H):
    """net_arch [H, H] (code/lorenz_pmsm/optimize.py:36-41 searches 64 and 128):
    zero-padded to the kernel's 128 units, the MFMA dataflow computes the narrow net."""
    net = pol.ActorCriticMlp(6, 2, hidden=H, seed=H)
    g = torch.Generator().manual_seed(H)
    with torch.no_grad():
        for p in net.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * (0.4 if p.dim() > 1 else 0.3))
    sd = {k: v.detach().clone() for k, v in net.state_dict().items()}
    blob = pol.pack_policy(sd, 6, 2)
    obs = np.random.default_rng(H).normal(0, 1.5, size=(32, 6)).astype(np.float32)
    mean, value = _emulate(pol, blob, obs)
    ref_mean, ref_value = pol.reference_forward_bf16(sd, obs)
    np.testing.assert_allclose(mean[:, :2], ref_mean.numpy(), rtol=0, atol=2e-4)
    np.testing.assert_allclose(value, ref_value.numpy(), rtol=0, atol=2e-4)
    from gym_lorenz import _native as nat
    big = pol.ActorCriticMlp(6, 2, hidden=129, seed=0).state_dict()
    with pytest.raises(nat.LorenzEnvError):
        pol.pack_policy(big, 6, 2)
