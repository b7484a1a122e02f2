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


def test_sb3_framestack_restatement_hand_case():
    from oracle.sb3_framestack import StackedObservations

    so = StackedObservations(2, 3, 2)
    st = so.reset(np.array([[1, 2], [3, 4]], np.float32))
    assert st.tolist() == [[0, 0, 0, 0, 1, 2], [0, 0, 0, 0, 3, 4]]
    infos = [{}, {"terminal_observation": np.array([9, 9], np.float32)}]
    st, infos = so.update(np.array([[5, 6], [7, 8]], np.float32), np.array([False, True]), infos)
    assert st.tolist() == [[0, 0, 1, 2, 5, 6], [0, 0, 0, 0, 7, 8]]
    assert infos[1]["terminal_observation"].tolist() == [0, 0, 3, 4, 9, 9]
