"""The opt-in "i8x4" policy precision on the host (no GPU): the oracle's restatement of the
split (lz_oracle.c orc_i8x_*, orc_attn_i8x4) against independent NumPy integer / float64
arithmetic, and its accuracy against the reference's own attention classes.

The scheme (lz_policy.hip attn16_net<kI8>): a float32 value v becomes the int32
V = rint(v 2^q), |V| <= 2^28, split into four balanced int8 digits (U = V + 0x808080; the
low three bytes of U ^ 0x80, the top byte of U); a dot product of two such vectors is the
sum of the 10 digit-pair products of levels i + j >= 3 -- exact int32 sums, which is what
v_mfma_i32_16x16x64_i8 computes, in any order -- recombined as
ldexpf(fmaf(float(L6 * 256 + L5), 2^16, float(L4 * 256 + L3)), 24 - q_w - q_v).
"""
import numpy as np
import pytest
import torch

F32 = np.float32


def _digits_np(V):
    U = (V.astype(np.int64) + 0x808080) & 0xFFFFFFFF
    U = np.where(U >= 1 << 31, U - (1 << 32), U)  # back to int32 two's complement
    lo = [(((U >> (8 * k)) & 0xFF) ^ 0x80).astype(np.uint8).view(np.int8) for k in range(3)]
    return np.stack(lo + [(U >> 24).astype(np.int8)], 1)


def test_digits_reconstruct_exactly(orc):
    rng = np.random.default_rng(0)
    v = np.concatenate([rng.uniform(-1, 1, 20000), [0.0, 1.0, -1.0, 1 - 2 ** -24, -0.5, 2 ** -30,
                                                    -2 ** -29, 0.999999]]).astype(F32)
    d = orc.i8x_digits(v, 28)
    V = np.rint(v.astype(np.float64) * 2.0 ** 28).astype(np.int64)
    assert np.array_equal(d, _digits_np(V))
    w = (2.0 ** (8 * np.arange(4)))[None, :]
    assert np.array_equal((d.astype(np.int64) * w.astype(np.int64)).sum(1), V)
    assert np.abs(d[:, 3].astype(int)).max() <= 16  # the top digit of |V| <= 2^28
    # a vector's scale: its largest magnitude m = f 2^e -> q = 28 - e, so |V| <= 2^28
    for m in (1.0, 0.75, 3.0, 1e-3, 200.0, 0.0):
        q = orc.i8x_row_q(np.array([m, -m / 3], F32))
        e = np.frexp(np.float32(m))[1] if m else 0
        assert q == 28 - e
        assert abs(np.rint(np.float64(m) * 2.0 ** q)) <= 2 ** 28


def _exact_level_dot(wd, vd):
    """the level-3..6 digit products in int64 and the recombination, independently"""
    L = np.zeros(7, np.int64)
    for i in range(4):
        for j in range(4):
            if i + j >= 3:
                L[i + j] += int((wd[:, i].astype(np.int64) * vd[:, j].astype(np.int64)).sum())
    return L


@pytest.mark.parametrize("K", [64, 128])
def test_dot_recombination_and_accuracy(orc, K):
    """orc_i8x_dot == the level sums done independently in int64 + the recombination; and
    its error against the exact dot product of the float32 inputs is that of float32's own
    k-ordered fmaf chain (what the f32 kernels compute): same worst case, lower median."""
    rng = np.random.default_rng(K)
    err_i8, err_f32 = [], []
    for trial in range(300):
        w = (rng.standard_normal(K) * rng.choice([1e-3, 0.05, 1.0, 30.0])).astype(F32)
        v = np.tanh(rng.standard_normal(K) * 2).astype(F32) if trial % 2 else \
            np.maximum(rng.standard_normal(K) * 5, 0).astype(F32)
        qw = orc.i8x_row_q(w)
        qv = orc.i8x_row_q(v) if trial % 2 == 0 else 28
        wd, vd = orc.i8x_digits(w, qw), orc.i8x_digits(v, qv)
        y = orc.i8x_dot(wd, vd, 24 - qw - qv)
        L = _exact_level_dot(wd, vd)
        hi, lo = L[6] * 256 + L[5], L[4] * 256 + L[3]
        assert abs(hi) < 2 ** 24 and abs(lo) < 2 ** 31  # the bounds the kernel relies on
        # fmaf(hi, 2^16, (float)lo): hi * 2^16 is exact, so one float32 rounding of the sum
        t = np.float32(np.float64(F32(hi)) * 65536.0 + np.float64(F32(lo)))
        assert y == np.ldexp(t, 24 - qw - qv), trial
        ex = float(np.dot(w.astype(np.float64), v.astype(np.float64)))
        scale = float(np.abs(w.astype(np.float64) * v.astype(np.float64)).sum()) or 1.0
        acc = F32(0.0)
        for k in range(K):  # float32 fmaf chain (fma == float64 product + sum, rounded once)
            acc = F32(np.float64(w[k]) * np.float64(v[k]) + np.float64(acc))
        err_i8.append(abs(float(y) - ex) / scale)
        err_f32.append(abs(float(acc) - ex) / scale)
    ei, ef = np.array(err_i8), np.array(err_f32)
    print("K=%d |y - exact| / sum|w v|: i8x4 max %.2e median %.2e; float32 fmaf chain max %.2e "
          "median %.2e" % (K, ei.max(), np.median(ei), ef.max(), np.median(ef)))
    assert ei.max() < 1.5 * ef.max() and np.median(ei) < np.median(ef)


def _attn_ref(tag):
    from conftest import golden

    g = golden("attn_ref")
    pre = tag + "/"
    sd = {k[len(pre):]: torch.from_numpy(v) for k, v in g.items()
          if k.startswith(pre) and k[len(pre):] not in ("x", "features", "mean", "value")}
    return sd, g[pre + "x"], g[pre + "features"], g[pre + "mean"], g[pre + "value"]


@pytest.mark.parametrize("tag", ["plain", "ln"])
def test_oracle_i8x4_vs_reference_classes(orc, tag):
    """VERDICT r04 #4's bar: the split oracle within 2e-6 (of the output scale) of the
    reference's own AttentionFeaturesExtractor classes (tests/golden/attn_ref.npz, torch
    float32), as the float32 oracle is; and within that of the float32 oracle itself."""
    sd, x, f_ref, m_ref, v_ref = _attn_ref(tag)
    m, v, f = orc.attn_f32(sd, x, return_features=True, precision="i8x4")
    m32, v32 = orc.attn_f32(sd, x)

    def rel(a, b):
        return float(np.abs(a - b).max() / max(1.0, np.abs(b).max()))

    dm, dv = rel(m, m_ref), rel(v, v_ref)
    print("orc_attn_i8x4 vs the reference's %s classes: mean %.2e, value %.2e (vs f32 oracle "
          "%.2e / %.2e)" % (tag, dm, dv, rel(m, m32), rel(v, v32)))
    assert rel(f, f_ref) < 2e-6  # (the extractor is orc_attn_f32's)
    assert dm < 2e-6 and dv < 2e-6
    assert rel(m, m32) < 2e-6 and rel(v, v32) < 2e-6


def test_oracle_i8x4_nonfinite_features(orc, pol):
    """A NaN or inf feature makes every output of that env NaN (and no other env's)."""
    net = pol.ActorCriticAttn(6, 2, seed=5)
    sd = net.state_dict()
    x = np.random.default_rng(1).standard_normal((6, 6)).astype(F32)
    x[1, 2] = np.nan
    x[4, 0] = np.inf
    m, v = orc.attn_f32(sd, x, precision="i8x4")
    m32, v32 = orc.attn_f32(sd, x)
    bad = ~np.isfinite(m32).all(1) | ~np.isfinite(v32)
    assert bad[1]
    assert np.isnan(m[bad]).all() and np.isnan(v[bad]).all()
    assert np.isfinite(m[~bad]).all() and np.isfinite(v[~bad]).all()


@pytest.fixture(scope="module")
def pol():
    from gym_lorenz import policy

    return policy


# ------------------------------------------------ the packed blob, read the kernel's way
PI, VF = 54400, 54400 + 102400          # lz_internal.h kAFPi / kAFVf
N1, N2, NB1, NB2, NH, NHB = 0, 32768, 98304, 98816, 99328, 101376
SH1, SH2 = NHB + 16, NHB + 16 + 256     # kAXSh1 / kAXSh2
POSTSH = SH2 + 256                      # kAXPostSh (pi slot)
POSTW, POSTB = 21376, 54144             # kAFPostW / kAFPostB (extractor)


def _lane_bytes(blob, off, n_ops):
    """[n_ops][64 lanes][16 B] int8 A operands at off"""
    return np.frombuffer(blob[off: off + n_ops * 64 * 16].tobytes(), np.int8).reshape(n_ops, 64, 16)


def _net_from_blob(orc, blob, base, feat, R):
    """attn16_net_i8 emulated from the packed bytes: lane (G, m) byte 4f + r of A operand
    (tile, [k-block,] digit) pairs with input 16f + 4G + r of the k-block; exact int64
    level sums; hi / lo recombined (float64 of hi * 2^16 + float32(lo) is exact, so one
    rounding to float32 == fmaf); the int16 row shifts; then bias, tanh_tab, heads."""
    b = blob.tobytes()
    n = feat.shape[0]
    sh1 = np.frombuffer(b[base + SH1: base + SH1 + 256], np.int16).astype(np.int64)
    sh2 = np.frombuffer(b[base + SH2: base + SH2 + 256], np.int16).astype(np.int64)
    f32 = lambda off, cnt: np.frombuffer(b[base + off: base + off + 4 * cnt], np.float32)  # noqa: E731
    b1, b2, wh, bh = f32(NB1, 128), f32(NB2, 128), f32(NH, 4 * 128).reshape(4, 128), f32(NHB, 4)
    m = np.max(feat, 1)
    qa = 28 - np.frexp(m.astype(np.float32))[1]

    def digits(v, q):  # [n, K] float32, q [n] -> [n, K, 4]
        return np.stack([orc.i8x_digits(v[i], q[i]) for i in range(v.shape[0])])

    def layer(x_d, ops, n_kb, sh, bias, qx):
        out = np.zeros((n, 128), np.float32)
        for t in range(8):
            for mm in range(16):
                u = 16 * t + mm
                L = np.zeros((n, 7), np.int64)
                for G in range(4):  # lane (G, mm) holds 16 of each k-block's 64 inputs
                    lane = 16 * G + mm
                    for kb in range(n_kb):
                        ks = np.array([64 * kb + 16 * f + 4 * G + r for f in range(4) for r in range(4)])
                        for i in range(4):
                            w = ops[(t * n_kb + kb) * 4 + i, lane].astype(np.int64)  # byte 4f + r
                            for j in range(4):
                                if i + j >= 3:
                                    L[:, i + j] += x_d[:, ks, j].astype(np.int64) @ w
                hi, lo = L[:, 6] * 256 + L[:, 5], L[:, 4] * 256 + L[:, 3]
                y = (np.float64(hi.astype(np.float32)) * 65536.0
                     + np.float64(lo.astype(np.float32))).astype(np.float32)
                y = np.ldexp(y, (sh[u] - qx).astype(np.int32)).astype(np.float32)
                out[:, u] = (y + bias[u]).astype(np.float32)
        return out

    fd = digits(feat, qa)
    a1 = orc.tanh_tab(layer(fd, _lane_bytes(blob, base + N1, 32), 1, sh1, b1, qa))
    ad = digits(a1, np.full(n, 28))
    a2 = orc.tanh_tab(layer(ad, _lane_bytes(blob, base + N2, 64), 2, sh2, b2, np.zeros(n, np.int64)))
    outs = []
    for r in range(R):
        part = []
        for G in range(4):
            acc = np.zeros(n, np.float32)
            for t in range(8):
                for c in range(4):
                    k = 16 * t + 4 * G + c
                    acc = (np.float64(wh[r, k]) * a2[:, k].astype(np.float64) + acc).astype(np.float32)
            part.append(acc)
        outs.append(((part[0] + part[1]) + (part[2] + part[3])) + bh[r])
    return np.stack(outs, 1)


@pytest.mark.parametrize("ln", [False, True])
def test_packed_blob_dataflow_equals_oracle(orc, pol, ln):
    """lz_attn[_ln]_policy_pack_i8x4's bytes, consumed in the kernel's lane / byte order
    (an emulation of v_mfma_i32_16x16x64_i8 over the blob), give the oracle's actions and
    values bit for bit: a wrong digit, byte or row-shift placement would not."""
    in_dim = 24 if ln else 6
    net = pol.ActorCriticAttn(in_dim, 2, seed=11, layer_norm=ln)
    g = torch.Generator().manual_seed(5)
    with torch.no_grad():
        for p in net.parameters():
            p.add_(torch.randn(p.shape, generator=g) * 0.05)
    sd = net.state_dict()
    pack = pol.pack_attn_ln_policy_i8x4 if ln else pol.pack_attn_policy_i8x4
    blob = pack(sd, in_dim, 2)
    x = np.random.default_rng(2).standard_normal((40, in_dim)).astype(F32) * 2
    m, v, feat = orc.attn_f32(sd, x, return_features=True, precision="i8x4")
    me = _net_from_blob(orc, blob, PI, feat, 2)
    ve = _net_from_blob(orc, blob, VF, feat, 1)[:, 0]
    assert np.array_equal(me.view(np.uint32), m.view(np.uint32))
    assert np.array_equal(ve.view(np.uint32), v.view(np.uint32))
    # post_attention_fc's digits (kAFPostW) and row shifts (the pi slot's kAXPostSh): byte
    # 4f + r of lane (G, m), A operand (tile u, k-block kb, digit i) = digit i of
    # post_w[16u + m][64kb + 16f + 4G + r] at its row's q
    post_w = sd["features_extractor.post_attention_fc.0.weight"].numpy()
    ops = _lane_bytes(blob, POSTW, 32)
    psh = np.frombuffer(blob[PI + POSTSH: PI + POSTSH + 128].tobytes(), np.int16)
    for row in range(64):
        q = orc.i8x_row_q(post_w[row])
        assert psh[row] == 24 - q
        dg = orc.i8x_digits(post_w[row], q)
        u, mm = row // 16, row % 16
        for G in range(4):
            for kb in range(2):
                ks = [64 * kb + 16 * f + 4 * G + r for f in range(4) for r in range(4)]
                for i in range(4):
                    assert np.array_equal(ops[(u * 2 + kb) * 4 + i, 16 * G + mm], dg[ks, i]), (row, G, kb, i)
    # the float32 blob differs only in those encodings and the shift tables
    b32 = (pol.pack_attn_ln_policy_f32 if ln else pol.pack_attn_policy_f32)(sd, in_dim, 2)
    same = np.ones(blob.size, bool)
    same[POSTW: POSTB] = False
    same[PI + POSTSH: PI + POSTSH + 128 + 16] = False  # shifts + the format tag (kAXTag)
    for base in (PI, VF):
        same[base + N1: base + NB1] = False
        same[base + SH1: base + SH2 + 256] = False
    assert np.array_equal(blob[same], b32[same])


@pytest.mark.parametrize("key", ["mlp_extractor.value_net.2.weight",
                                 "features_extractor.post_attention_fc.0.weight"])
def test_pack_refuses_nonfinite_weights(pol, key):
    from gym_lorenz import _native as nat

    sd = pol.ActorCriticAttn(6, 2, seed=1).state_dict()
    sd[key][3, 7] = float("inf")
    with pytest.raises(nat.LorenzEnvError):
        pol.pack_attn_policy_i8x4(sd, 6, 2)
