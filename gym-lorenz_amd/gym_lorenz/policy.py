"""Policy in the loop: SB3 on-policy rollout collection fused on the GPU.

The reference trains its envs with stable-baselines3 A2C / PPO ``"MlpPolicy"``
actor-critics, ``net_arch=dict(pi=[128, 128], vf=[128, 128])`` with Tanh
(code/lorenz_pmsm/train.py:155-178: A2C, n_steps=16, VecNormalize(norm_obs=True,
norm_reward=False, clip_obs=10); code/lorenz_filter/train.py:117-127 and
code/gym_try.py:106-116: PPO, n_steps=2048, gae_lambda=0.95; code/gym_run.py:79).
SB3 then runs ``OnPolicyAlgorithm.collect_rollouts``: per step one policy forward on
the host, one ``DummyVecEnv.step`` over the envs one at a time, a RolloutBuffer add,
and finally ``RolloutBuffer.compute_returns_and_advantage``.

``FusedRolloutCollector.collect(K)`` does all K steps in ONE kernel launch
(``lz_rollout_policy_f32``): the two 6->128->128 MLPs at SB3's own precision
(float32 operands and accumulation on f32-input MFMA, a deterministic operation order
the C oracle reproduces bit for bit -- likewise code/train.py's and code/lorenz_filter/
train.py's attention actor-critics, ``lz_rollout_policy_attn_f32`` / ``_attn_stack_f32``;
``precision="bf16"`` selects the faster bf16-MFMA kernels), the Gaussian
sample (Philox), the action-space clip, the env step with
auto-reset, SB3's truncation bootstrap, and VecNormalize's observation normalisation.
With a training VecNormalize the float32 kernel follows SB3's order exactly: each
step's batch updates obs_rms before that step's observations are normalised
(``lz_rollout_policy_f32_vn``: one launch per step, the statistics update between
launches); ``vecnorm_update="rollout"`` (and the bf16 / attention kernels) keep the
statistics frozen for the K steps and update them once from the pooled moments.
``compute_returns_and_advantage`` is ``lz_gae``.  The buffers come back as
time-major device tensors in SB3's RolloutBuffer layout ([K, N, ...]).

``ActorCriticMlp`` is a plain-torch restatement of SB3's ActorCriticPolicy for this
net_arch (same state_dict keys, same orthogonal init) -- the weight source when SB3 is
absent and the fp32 reference in the tests.  An SB3 policy's ``state_dict()`` can be
passed to ``set_params`` directly.
"""
import ctypes
import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist
from torch import nn

from . import _native as nat
from .registry import LEGACY_SPECS, SPECS

HIDDEN = nat.POLICY_HIDDEN

KEYS = ("mlp_extractor.policy_net.0.weight", "mlp_extractor.policy_net.0.bias",
        "mlp_extractor.policy_net.2.weight", "mlp_extractor.policy_net.2.bias",
        "mlp_extractor.value_net.0.weight", "mlp_extractor.value_net.0.bias",
        "mlp_extractor.value_net.2.weight", "mlp_extractor.value_net.2.bias",
        "action_net.weight", "action_net.bias", "value_net.weight", "value_net.bias", "log_std")
_FIELDS = ("pi_w1", "pi_b1", "pi_w2", "pi_b2", "vf_w1", "vf_b1", "vf_w2", "vf_b2",
           "act_w", "act_b", "val_w", "val_b", "log_std")


def action_bounds(system_name):
    for spec in list(SPECS.values()) + list(LEGACY_SPECS.values()):
        if spec.system_name == system_name:
            return float(spec.act[0]), float(spec.act[1])
    raise KeyError(system_name)


class _MlpExtractor(nn.Module):
    def __init__(self, obs_dim, hidden=HIDDEN):
        super().__init__()
        self.policy_net = nn.Sequential(nn.Linear(obs_dim, hidden), nn.Tanh(),
                                        nn.Linear(hidden, hidden), nn.Tanh())
        self.value_net = nn.Sequential(nn.Linear(obs_dim, hidden), nn.Tanh(),
                                       nn.Linear(hidden, hidden), nn.Tanh())


class ActorCriticMlp(nn.Module):
    """SB3 ActorCriticPolicy (MlpPolicy, net_arch pi=[128,128] vf=[128,128], Tanh,
    DiagGaussian, log_std_init=0, ortho_init=True) in plain torch, fp32."""

    def __init__(self, obs_dim, act_dim, hidden=HIDDEN, log_std_init=0.0, seed=None):
        super().__init__()
        g = torch.Generator().manual_seed(seed) if seed is not None else None
        self.mlp_extractor = _MlpExtractor(obs_dim, hidden)
        self.action_net = nn.Linear(hidden, act_dim)
        self.value_net = nn.Linear(hidden, 1)
        self.log_std = nn.Parameter(torch.ones(act_dim) * log_std_init)
        # SB3 ActorCriticPolicy._build: orthogonal init, gains sqrt(2) / 0.01 / 1, zero bias
        with torch.no_grad():
            for mod, gain in ((self.mlp_extractor, math.sqrt(2)), (self.action_net, 0.01),
                              (self.value_net, 1.0)):
                for m in mod.modules():
                    if isinstance(m, nn.Linear):
                        nn.init.orthogonal_(m.weight, gain=gain, generator=g)
                        m.bias.zero_()

    def forward(self, obs):
        """(mean actions, values) in fp32."""
        mean = self.action_net(self.mlp_extractor.policy_net(obs))
        value = self.value_net(self.mlp_extractor.value_net(obs)).flatten()
        return mean, value


class AttentionFeaturesExtractor(nn.Module):
    """code/train.py:52-95 restated in plain torch (same submodule names, so the same
    state_dict keys under ``features_extractor.``): fc1 obs->128 + ReLU, the 128 units
    as 8 tokens of 16, nn.MultiheadAttention(16, 4 heads, batch_first) self-attention,
    flatten, post_attention_fc 128->features_dim + ReLU."""

    def __init__(self, obs_dim, features_dim=64):
        super().__init__()
        self.hidden_dim, self.seq_len, self.token_dim = 128, 8, 16
        self.features_dim = features_dim
        self.fc1 = nn.Linear(obs_dim, self.hidden_dim)
        self.attention_layer = nn.MultiheadAttention(embed_dim=self.token_dim, num_heads=4,
                                                     batch_first=True)
        self.post_attention_fc = nn.Sequential(nn.Linear(self.hidden_dim, features_dim), nn.ReLU())

    def forward(self, observations):
        x = torch.relu(self.fc1(observations))
        x_seq = x.view(-1, self.seq_len, self.token_dim)
        attn_output, _ = self.attention_layer(x_seq, x_seq, x_seq)
        return self.post_attention_fc(attn_output.reshape(-1, self.hidden_dim))


class AttentionFeaturesExtractorLN(AttentionFeaturesExtractor):
    """code/lorenz_filter/train.py:54-103: the same extractor with a residual connection
    and LayerNorm(16) per token after the attention (x_seq = layer_norm(x_seq +
    attn_output)) before post_attention_fc; used there on VecFrameStack(n_stack=4)."""

    def __init__(self, obs_dim, features_dim=64):
        super().__init__(obs_dim, features_dim)
        self.layer_norm = nn.LayerNorm(self.token_dim)

    def forward(self, observations):
        x = torch.relu(self.fc1(observations))
        x_seq = x.view(-1, self.seq_len, self.token_dim)
        attn_output, _ = self.attention_layer(x_seq, x_seq, x_seq)
        x_seq = self.layer_norm(x_seq + attn_output)
        return self.post_attention_fc(x_seq.reshape(-1, self.hidden_dim))


class ActorCriticAttn(nn.Module):
    """SB3 ActorCriticPolicy as code/train.py:101-112 builds it: the shared
    AttentionFeaturesExtractor (features_dim=64), net_arch pi=[128,128] vf=[128,128]
    Tanh, DiagGaussian (log_std_init=0), SB3's orthogonal init (gain sqrt(2) for the
    extractor and the nets, 0.01 / 1 for the heads, zero biases; init_weights touches
    nn.Linear modules only, so in_proj keeps torch's xavier init)."""

    def __init__(self, obs_dim, act_dim, features_dim=64, hidden=HIDDEN, log_std_init=0.0,
                 seed=None, layer_norm=False):
        super().__init__()
        g = torch.Generator().manual_seed(seed) if seed is not None else None
        if seed is not None:
            torch.manual_seed(seed)  # nn.MultiheadAttention's own xavier init
        ext = AttentionFeaturesExtractorLN if layer_norm else AttentionFeaturesExtractor
        self.features_extractor = ext(obs_dim, features_dim)
        self.mlp_extractor = _MlpExtractor(features_dim, hidden)
        self.action_net = nn.Linear(hidden, act_dim)
        self.value_net = nn.Linear(hidden, 1)
        self.log_std = nn.Parameter(torch.ones(act_dim) * log_std_init)
        with torch.no_grad():
            for mod, gain in ((self.features_extractor, math.sqrt(2)),
                              (self.mlp_extractor, math.sqrt(2)), (self.action_net, 0.01),
                              (self.value_net, 1.0)):
                for m in mod.modules():
                    if isinstance(m, nn.Linear):
                        nn.init.orthogonal_(m.weight, gain=gain, generator=g)
                        m.bias.zero_()

    def forward(self, obs):
        f = self.features_extractor(obs)
        mean = self.action_net(self.mlp_extractor.policy_net(f))
        value = self.value_net(self.mlp_extractor.value_net(f)).flatten()
        return mean, value


def _bf(t):
    return t.to(torch.bfloat16).to(torch.float32)


# 2 / ln 2 in float32: lz_policy_pack stores the two tanh layers as bf16(s * W) and
# s * b so that the kernel's tanh needs no multiply (lz_policy.hip tanh_scaled)
TANH_SCALE = np.float32(2.8853900817779268)


def reference_forward_bf16(state_dict, obs):
    """The fused kernel's arithmetic restated in torch: bf16 operands (the tanh layers'
    weights as bf16(s W) with s = 2/ln 2 folded in, the head's as bf16(W), and each
    layer's input activations rounded to bf16, round-to-nearest-even), fp32 bias and
    accumulation, tanh(acc / s).  Differs from the kernel only in fp32 summation order
    and the tanh implementation (|err| <= 2e-7).  Returns (mean, value)."""
    sd = {k: torch.as_tensor(np.asarray(_np(v)), dtype=torch.float32) for k, v in state_dict.items()}
    x = _bf(torch.as_tensor(obs, dtype=torch.float32))
    s = torch.tensor(TANH_SCALE)

    def net(prefix, w3, b3):
        h = x
        for layer in (".0", ".2"):
            acc = h @ _bf(s * sd[prefix + layer + ".weight"]).T + s * sd[prefix + layer + ".bias"]
            h = _bf(torch.tanh(acc / s))
        return h @ _bf(sd[w3]).T + sd[b3]

    mean = net("mlp_extractor.policy_net", "action_net.weight", "action_net.bias")
    value = net("mlp_extractor.value_net", "value_net.weight", "value_net.bias").flatten()
    return mean, value


# log2(e) / sqrt(head dim 4): lz_attn_policy_pack stores the Q projection pre-scaled by
# it (bf16(c W_q), c b_q) so the kernel's softmax is exp2(q.k - max)
ATTN_Q_SCALE = 1.4426950408889634 / 2.0
FE = "features_extractor."
ATTN_FE_KEYS = ("fc1.weight", "fc1.bias", "attention_layer.in_proj_weight",
                "attention_layer.in_proj_bias", "attention_layer.out_proj.weight",
                "attention_layer.out_proj.bias", "post_attention_fc.0.weight",
                "post_attention_fc.0.bias")
_ATTN_FE_FIELDS = ("fc1_w", "fc1_b", "in_proj_w", "in_proj_b", "out_proj_w", "out_proj_b",
                   "post_w", "post_b")


def is_attention_policy(state_dict):
    """True for a state_dict of code/train.py's AttentionFeaturesExtractor policy."""
    return any(k.endswith("features_extractor.fc1.weight") for k in state_dict)


def is_attention_ln_policy(state_dict):
    """True for code/lorenz_filter/train.py's residual + LayerNorm extractor."""
    return any(k.endswith("features_extractor.layer_norm.weight") for k in state_dict)


def _fe_key(state_dict, name):
    # SB3 (share_features_extractor=True) stores the shared extractor under
    # features_extractor. and aliases it as pi_features_extractor. / vf_features_extractor.
    for pre in (FE, "pi_" + FE):
        if pre + name in state_dict:
            return pre + name
    raise KeyError("policy state_dict lacks %r (expected code/train.py's "
                   "AttentionFeaturesExtractor)" % (FE + name))


def attn_folded_post(sd):
    """out_proj folded into post_attention_fc, float64 (as lz_attn_policy_pack):
    Wf [8 tokens, 64, 16] and the folded bias [64]."""
    g = {k: torch.as_tensor(np.asarray(_np(sd[_fe_key(sd, k)])), dtype=torch.float64)
         for k in ATTN_FE_KEYS[4:]}
    wo, bo = g["attention_layer.out_proj.weight"], g["attention_layer.out_proj.bias"]
    wp, bp = g["post_attention_fc.0.weight"], g["post_attention_fc.0.bias"]
    blocks = wp.view(wp.shape[0], 8, 16).permute(1, 0, 2)  # [8, 64, 16]
    wf = blocks @ wo
    bf = bp + (blocks @ bo).sum(0)
    return wf, bf


def reference_forward_attn_bf16(state_dict, obs):
    """lz_rollout_policy_attn's arithmetic restated in torch: bf16 obs / weights /
    tokens / head outputs / features (RNE), fp32 accumulation and attention, the Q
    projection pre-scaled by ATTN_Q_SCALE and a base-2 softmax, out_proj folded into
    post_attention_fc in float64, the Tanh nets as reference_forward_bf16.  Differs
    from the kernel in fp32 summation order and the exp2 / rcp / tanh implementations.
    Returns (mean, value)."""
    sd = state_dict
    f32 = torch.float32

    def t(k):
        return torch.as_tensor(np.asarray(_np(sd[k])), dtype=f32)

    x = _bf(torch.as_tensor(obs, dtype=f32))
    n = x.shape[0]
    tok = _bf(torch.relu(x @ _bf(t(_fe_key(sd, "fc1.weight"))).T + t(_fe_key(sd, "fc1.bias"))))
    tok = tok.view(n, 8, 16)
    w_in, b_in = t(_fe_key(sd, ATTN_FE_KEYS[2])), t(_fe_key(sd, ATTN_FE_KEYS[3]))
    c = torch.tensor(np.float64(ATTN_Q_SCALE))
    wq = _bf((c.double() * w_in[:16].double()).to(f32))
    bq = (c.double() * b_in[:16].double()).to(f32)
    q = tok @ wq.T + bq
    k = tok @ _bf(w_in[16:32]).T + b_in[16:32]
    v = tok @ _bf(w_in[32:48]).T + b_in[32:48]
    q, k, v = (z.view(n, 8, 4, 4).transpose(1, 2) for z in (q, k, v))  # [n, head, token, 4]
    s = q @ k.transpose(-1, -2)
    p = torch.exp2(s - s.amax(-1, keepdim=True))
    o = (p @ v) * (1.0 / p.sum(-1, keepdim=True))  # normalised after the weighted sum
    a = _bf(o.transpose(1, 2).reshape(n, 8, 16))
    wf, bfold = attn_folded_post(sd)
    feat = bfold.to(f32) + torch.einsum("nid,ifd->nf", a, _bf(wf.to(f32)))
    feat = _bf(torch.relu(feat))
    s_t = torch.tensor(TANH_SCALE)

    def net(prefix, w3, b3):
        h = feat
        for layer in (".0", ".2"):
            acc = h @ _bf(s_t * t(prefix + layer + ".weight")).T + s_t * t(prefix + layer + ".bias")
            h = _bf(torch.tanh(acc / s_t))
        return h @ _bf(t(w3)).T + t(b3)

    mean = net("mlp_extractor.policy_net", "action_net.weight", "action_net.bias")
    value = net("mlp_extractor.value_net", "value_net.weight", "value_net.bias").flatten()
    return mean, value


def reference_forward_attn_ln_bf16(state_dict, obs):
    """lz_rollout_policy_attn_stack's arithmetic restated in torch (code/lorenz_filter/
    train.py's extractor): as reference_forward_attn_bf16 up to the head outputs, then
    out_proj (bf16 operands, fp32 accumulate), the residual with the bf16 token values,
    LayerNorm(16) in fp32 (biased variance, eps 1e-5), bf16, post_attention_fc (bf16
    operands) + ReLU, the Tanh nets.  obs: the (stacked) policy input.  Returns
    (mean, value)."""
    sd = state_dict
    f32 = torch.float32

    def t(k):
        return torch.as_tensor(np.asarray(_np(sd[k])), dtype=f32)

    x = _bf(torch.as_tensor(obs, dtype=f32))
    n = x.shape[0]
    tok = _bf(torch.relu(x @ _bf(t(_fe_key(sd, "fc1.weight"))).T + t(_fe_key(sd, "fc1.bias"))))
    tok = tok.view(n, 8, 16)
    w_in, b_in = t(_fe_key(sd, ATTN_FE_KEYS[2])), t(_fe_key(sd, ATTN_FE_KEYS[3]))
    c = torch.tensor(np.float64(ATTN_Q_SCALE))
    wq = _bf((c.double() * w_in[:16].double()).to(f32))
    bq = (c.double() * b_in[:16].double()).to(f32)
    q = tok @ wq.T + bq
    k = tok @ _bf(w_in[16:32]).T + b_in[16:32]
    v = tok @ _bf(w_in[32:48]).T + b_in[32:48]
    q, k, v = (z.view(n, 8, 4, 4).transpose(1, 2) for z in (q, k, v))
    s = q @ k.transpose(-1, -2)
    p = torch.exp2(s - s.amax(-1, keepdim=True))
    o = (p @ v) * (1.0 / p.sum(-1, keepdim=True))
    a = _bf(o.transpose(1, 2).reshape(n, 8, 16))
    y = a @ _bf(t(_fe_key(sd, ATTN_FE_KEYS[4]))).T + t(_fe_key(sd, ATTN_FE_KEYS[5]))
    z = y + tok
    mu = z.mean(-1, keepdim=True)
    z = z - mu
    var = (z * z).mean(-1, keepdim=True)
    u = _bf(z * torch.rsqrt(var + 1e-5) * t(_fe_key(sd, "layer_norm.weight"))
            + t(_fe_key(sd, "layer_norm.bias")))
    feat = _bf(torch.relu(u.reshape(n, 128) @ _bf(t(_fe_key(sd, ATTN_FE_KEYS[6]))).T
                          + t(_fe_key(sd, ATTN_FE_KEYS[7]))))
    s_t = torch.tensor(TANH_SCALE)

    def net(prefix, w3, b3):
        h = feat
        for layer in (".0", ".2"):
            acc = h @ _bf(s_t * t(prefix + layer + ".weight")).T + s_t * t(prefix + layer + ".bias")
            h = _bf(torch.tanh(acc / s_t))
        return h @ _bf(t(w3)).T + t(b3)

    mean = net("mlp_extractor.policy_net", "action_net.weight", "action_net.bias")
    value = net("mlp_extractor.value_net", "value_net.weight", "value_net.bias").flatten()
    return mean, value


def _np(v):
    if isinstance(v, torch.Tensor):
        return v.detach().to("cpu", torch.float32).numpy()
    return np.asarray(v, np.float32)


def _mlp_policy_struct(state_dict, obs_dim, act_dim):
    arrs = []
    for key in KEYS:
        if key not in state_dict:
            raise KeyError("policy state_dict lacks %r (expected SB3 MlpPolicy with "
                           "net_arch pi=[H,H] vf=[H,H], H <= 128)" % key)
        arrs.append(np.ascontiguousarray(_np(state_dict[key]), dtype=np.float32))
    H = arrs[0].shape[0]
    shapes = [(H, obs_dim), (H,), (H, H), (H,)] * 2 + [
        (act_dim, H), (act_dim,), (1, H), (1,), (act_dim,)]
    for key, a, shp in zip(KEYS, arrs, shapes):
        if a.shape != shp:
            raise ValueError("%s has shape %s, expected %s" % (key, a.shape, shp))
    p = nat.LzMlpPolicy()
    p.obs_dim, p.act_dim = int(obs_dim), int(act_dim)
    for f, a in zip(_FIELDS, arrs):
        setattr(p, f, a.ctypes.data)
    return p, H, arrs  # arrs keep the weights alive while p points at them


def pack_policy_f32(state_dict, obs_dim, act_dim):
    """lz_policy_pack_f32: SB3 state_dict (net_arch pi=[H,H] vf=[H,H], H <= 128) ->
    uint8 numpy blob of the float32 kernel (host; needs no GPU)."""
    p, H, _keep = _mlp_policy_struct(state_dict, obs_dim, act_dim)
    blob = np.zeros(int(nat.lib.lz_policy_f32_blob_bytes()), np.uint8)
    nat.check(nat.lib.lz_policy_pack_f32(ctypes.byref(p), H, blob.ctypes.data, blob.size))
    return blob


def pack_policy_i8x4(state_dict, obs_dim, act_dim):
    """lz_policy_pack_i8x4: the float32 MlpPolicy blob with each net's layer 2 as exact
    4-digit int8 fixed-point products (precision="i8x4"; oracle orc_mlp_i8x4)."""
    p, H, _keep = _mlp_policy_struct(state_dict, obs_dim, act_dim)
    blob = np.zeros(int(nat.lib.lz_policy_f32_blob_bytes()), np.uint8)
    nat.check(nat.lib.lz_policy_pack_i8x4(ctypes.byref(p), H, blob.ctypes.data, blob.size))
    return blob


def pack_policy(state_dict, obs_dim, act_dim):
    """lz_policy_pack / lz_policy_pack_hidden: SB3 state_dict (net_arch pi=[H,H]
    vf=[H,H], H <= 128) -> uint8 numpy blob of the bf16 kernel (host; needs no GPU)."""
    p, H, _keep = _mlp_policy_struct(state_dict, obs_dim, act_dim)
    blob = np.zeros(int(nat.lib.lz_policy_blob_bytes()), np.uint8)
    nat.check(nat.lib.lz_policy_pack_hidden(ctypes.byref(p), H, blob.ctypes.data, blob.size))
    return blob


def _attn_struct(state_dict, in_dim, act_dim, features_dim, ln):
    if features_dim != 64:
        raise ValueError("the fused kernel implements features_dim=64 (code/train.py:100)")
    keys = [_fe_key(state_dict, k) for k in ATTN_FE_KEYS] + list(KEYS)
    if ln:
        keys += [_fe_key(state_dict, "layer_norm.weight"), _fe_key(state_dict, "layer_norm.bias")]
    for key in KEYS:
        if key not in state_dict:
            raise KeyError("policy state_dict lacks %r" % key)
    arrs = [np.ascontiguousarray(_np(state_dict[k]), dtype=np.float32) for k in keys]
    F = features_dim
    shapes = [(HIDDEN, in_dim), (HIDDEN,), (48, 16), (48,), (16, 16), (16,), (F, HIDDEN), (F,)] + [
        (HIDDEN, F), (HIDDEN,), (HIDDEN, HIDDEN), (HIDDEN,)] * 2 + [
        (act_dim, HIDDEN), (act_dim,), (1, HIDDEN), (1,), (act_dim,)] + ([(16,), (16,)] if ln else [])
    for key, a, shp in zip(keys, arrs, shapes):
        if a.shape != shp:
            raise ValueError("%s has shape %s, expected %s" % (key, a.shape, shp))
    p = nat.LzAttnPolicy()
    p.obs_dim, p.act_dim = int(in_dim), int(act_dim)
    for f, a in zip(_ATTN_FE_FIELDS + _FIELDS, arrs):
        setattr(p, f, a.ctypes.data)
    if not ln:
        return p, arrs
    q = nat.LzAttnLnPolicy()
    q.attn = p
    q.ln_w, q.ln_b = arrs[-2].ctypes.data, arrs[-1].ctypes.data
    return q, arrs


def pack_attn_policy_f32(state_dict, obs_dim, act_dim, features_dim=64):
    """lz_attn_policy_pack_f32: code/train.py's attention actor-critic at SB3's float32
    precision (lz_rollout_policy_attn_f32) -> uint8 numpy blob (host; needs no GPU)."""
    p, _keep = _attn_struct(state_dict, obs_dim, act_dim, features_dim, False)
    blob = np.zeros(int(nat.lib.lz_attn_policy_f32_blob_bytes()), np.uint8)
    nat.check(nat.lib.lz_attn_policy_pack_f32(ctypes.byref(p), blob.ctypes.data, blob.size))
    return blob


def pack_attn_ln_policy_f32(state_dict, in_dim, act_dim, features_dim=64):
    """lz_attn_ln_policy_pack_f32: code/lorenz_filter/train.py's residual + LayerNorm
    policy at float32 precision (in_dim = the stacked observation width)."""
    p, _keep = _attn_struct(state_dict, in_dim, act_dim, features_dim, True)
    blob = np.zeros(int(nat.lib.lz_attn_policy_f32_blob_bytes()), np.uint8)
    nat.check(nat.lib.lz_attn_ln_policy_pack_f32(ctypes.byref(p), blob.ctypes.data, blob.size))
    return blob


def pack_attn_policy_i8x4(state_dict, obs_dim, act_dim, features_dim=64):
    """lz_attn_policy_pack_i8x4: code/train.py's attention actor-critic with the nets' two
    wide layers as exact 4-digit int8 fixed-point products (precision="i8x4"; the float32
    blob's size and layout otherwise) -> uint8 numpy blob (host; needs no GPU)."""
    p, _keep = _attn_struct(state_dict, obs_dim, act_dim, features_dim, False)
    blob = np.zeros(int(nat.lib.lz_attn_policy_f32_blob_bytes()), np.uint8)
    nat.check(nat.lib.lz_attn_policy_pack_i8x4(ctypes.byref(p), blob.ctypes.data, blob.size))
    return blob


def pack_attn_ln_policy_i8x4(state_dict, in_dim, act_dim, features_dim=64):
    """lz_attn_ln_policy_pack_i8x4: code/lorenz_filter/train.py's residual + LayerNorm
    policy, precision="i8x4" (in_dim = the stacked observation width)."""
    p, _keep = _attn_struct(state_dict, in_dim, act_dim, features_dim, True)
    blob = np.zeros(int(nat.lib.lz_attn_policy_f32_blob_bytes()), np.uint8)
    nat.check(nat.lib.lz_attn_ln_policy_pack_i8x4(ctypes.byref(p), blob.ctypes.data, blob.size))
    return blob


def pack_attn_policy(state_dict, obs_dim, act_dim, features_dim=64):
    """lz_attn_policy_pack: SB3 state_dict of code/train.py's attention actor-critic ->
    uint8 numpy blob (host; needs no GPU)."""
    if features_dim != 64:
        raise ValueError("the fused kernel implements features_dim=64 (code/train.py:100)")
    keys = [_fe_key(state_dict, k) for k in ATTN_FE_KEYS] + list(KEYS)
    for key in KEYS:
        if key not in state_dict:
            raise KeyError("policy state_dict lacks %r" % key)
    arrs = [np.ascontiguousarray(_np(state_dict[k]), dtype=np.float32) for k in keys]
    F = features_dim
    shapes = [(HIDDEN, obs_dim), (HIDDEN,), (48, 16), (48,), (16, 16), (16,), (F, HIDDEN), (F,)] + [
        (HIDDEN, F), (HIDDEN,), (HIDDEN, HIDDEN), (HIDDEN,)] * 2 + [
        (act_dim, HIDDEN), (act_dim,), (1, HIDDEN), (1,), (act_dim,)]
    for key, a, shp in zip(keys, arrs, shapes):
        if a.shape != shp:
            raise ValueError("%s has shape %s, expected %s" % (key, a.shape, shp))
    p = nat.LzAttnPolicy()
    p.obs_dim, p.act_dim = int(obs_dim), int(act_dim)
    for f, a in zip(_ATTN_FE_FIELDS + _FIELDS, arrs):
        setattr(p, f, a.ctypes.data)
    blob = np.zeros(int(nat.lib.lz_attn_policy_blob_bytes()), np.uint8)
    nat.check(nat.lib.lz_attn_policy_pack(ctypes.byref(p), blob.ctypes.data, blob.size))
    return blob


def pack_attn_ln_policy(state_dict, in_dim, act_dim, features_dim=64):
    """lz_attn_ln_policy_pack: code/lorenz_filter/train.py's policy (in_dim = the
    stacked observation width) -> uint8 numpy blob (host; needs no GPU)."""
    if features_dim != 64:
        raise ValueError("the fused kernel implements features_dim=64")
    keys = [_fe_key(state_dict, k) for k in ATTN_FE_KEYS] + list(KEYS) + [
        _fe_key(state_dict, "layer_norm.weight"), _fe_key(state_dict, "layer_norm.bias")]
    for key in KEYS:
        if key not in state_dict:
            raise KeyError("policy state_dict lacks %r" % key)
    arrs = [np.ascontiguousarray(_np(state_dict[k]), dtype=np.float32) for k in keys]
    F = features_dim
    shapes = [(HIDDEN, in_dim), (HIDDEN,), (48, 16), (48,), (16, 16), (16,), (F, HIDDEN), (F,)] + [
        (HIDDEN, F), (HIDDEN,), (HIDDEN, HIDDEN), (HIDDEN,)] * 2 + [
        (act_dim, HIDDEN), (act_dim,), (1, HIDDEN), (1,), (act_dim,), (16,), (16,)]
    for key, a, shp in zip(keys, arrs, shapes):
        if a.shape != shp:
            raise ValueError("%s has shape %s, expected %s" % (key, a.shape, shp))
    p = nat.LzAttnLnPolicy()
    p.attn.obs_dim, p.attn.act_dim = int(in_dim), int(act_dim)
    for f, a in zip(_ATTN_FE_FIELDS + _FIELDS, arrs):
        setattr(p.attn, f, a.ctypes.data)
    p.ln_w, p.ln_b = arrs[-2].ctypes.data, arrs[-1].ctypes.data
    blob = np.zeros(int(nat.lib.lz_attn_ln_policy_blob_bytes()), np.uint8)
    nat.check(nat.lib.lz_attn_ln_policy_pack(ctypes.byref(p), blob.ctypes.data, blob.size))
    return blob


@dataclass
class RolloutBatch:
    """SB3 RolloutBuffer contents, time-major device tensors."""
    observations: torch.Tensor   # [K, N, O] what the policy saw (normalised)
    actions: torch.Tensor        # [K, N, A] unclipped samples
    log_probs: torch.Tensor      # [K, N]
    values: torch.Tensor         # [K, N]
    rewards: torch.Tensor        # [K, N] (+ gamma * V(terminal obs) on truncation)
    dones: torch.Tensor          # [K, N] uint8 LZ_DONE_* bits of each step
    episode_starts: torch.Tensor  # [K, N] float32 (SB3 _last_episode_starts per step)
    last_values: torch.Tensor    # [N] V(normalised last obs)
    last_obs: torch.Tensor       # [N, O] raw
    obs_moments: torch.Tensor = None  # [1 + 2 O] float64 or None
    done_idx: torch.Tensor = None     # compact list k*N + env
    terminal_obs: torch.Tensor = None
    n_done: torch.Tensor = None
    last_stack: torch.Tensor = None   # [N, n_stack * O] VecFrameStack obs after the rollout
    advantages: torch.Tensor = None
    returns: torch.Tensor = None


def _p(t):
    return None if t is None else t.data_ptr()


def blob_format(attention, attention_ln, i8x4):
    """The LZ_BLOB_* format a float32 / i8x4 launch reads (entry point + LZ_POLICY_I8X4)."""
    if attention_ln:
        return nat.BLOB_ATTN_LN_I8X4 if i8x4 else nat.BLOB_ATTN_LN_F32
    if attention:
        return nat.BLOB_ATTN_I8X4 if i8x4 else nat.BLOB_ATTN_F32
    return nat.BLOB_MLP_I8X4 if i8x4 else nat.BLOB_MLP_F32


class FusedRolloutCollector:
    """OnPolicyAlgorithm.collect_rollouts over a BatchedEnv, one launch per rollout.

    backend:       gym_lorenz.core.BatchedEnv (float32, autoreset)
    state_dict:    SB3 ActorCriticPolicy / ActorCriticMlp state_dict
    obs_rms:       gym_lorenz.vec_normalize.DeviceRunningMeanStd or None
    training:      update obs_rms (VecNormalize.training)
    vecnorm_update: how a training obs_rms is updated.  "step" (the default for the
                   float32 MlpPolicy): SB3's order -- every step's batch updates obs_rms
                   before that step's observations (and the truncated steps' terminal
                   observations) are normalised (lz_rollout_policy_f32_vn: one launch
                   per step + the statistics update between).  "rollout" (opt-in; the
                   only mode of the bf16 / attention kernels): the K steps run in one
                   launch with the rollout-start statistics and one update from the K
                   steps' pooled moments afterwards -- faster, not SB3's trajectory.
    precision:     policy arithmetic: "fp32" (default; SB3's float32 forward --
                   lz_rollout_policy_f32, and for the attention actor-critics of
                   code/train.py / code/lorenz_filter/train.py lz_rollout_policy_attn_f32 /
                   _attn_stack_f32), "i8x4" (the same float32 kernels with the pi / vf
                   nets' wide layers as exact 4-digit int8 fixed-point products on the
                   int8 MFMA -- float32-level accuracy, bit-exact vs orc_attn_i8x4 /
                   orc_mlp_i8x4, not bit-equal to "fp32"; the MlpPolicy one without the
                   per-step VecNormalize collect, and for LORENZ3 / LORENZ4 / PMSM / HR)
                   or "bf16" (bf16 MFMA
                   operands, fp32 accumulation: lz_rollout_policy / _attn / _attn_stack,
                   ~2.5-5x faster, ~1e-2 off SB3).
    """

    def __init__(self, backend, state_dict=None, gamma=0.99, gae_lambda=0.95, obs_rms=None,
                 clip_obs=10.0, norm_eps=1e-8, training=True, bootstrap=True,
                 deterministic=False, capture_terminal=0, group=None, frame_stack=1,
                 precision=None, vecnorm_update=None):
        if backend.tdtype != torch.float32:
            raise ValueError("the fused policy rollout runs float32 env handles")
        self.env = backend
        self.device = backend.device
        self.n, self.O, self.A = backend.num_envs, backend.obs_dim, backend.action_dim
        self.gamma, self.gae_lambda = float(gamma), float(gae_lambda)
        self.obs_rms, self.clip_obs, self.norm_eps = obs_rms, float(clip_obs), float(norm_eps)
        self.training, self.bootstrap, self.deterministic = training, bootstrap, deterministic
        self.capture_terminal = int(capture_terminal)
        self.group = group
        self.act_low, self.act_high = action_bounds(backend.system_name)
        if precision not in (None, "fp32", "bf16", "i8x4"):
            raise ValueError("precision must be 'fp32', 'i8x4' or 'bf16'")
        self.precision = precision
        if vecnorm_update not in (None, "step", "rollout"):
            raise ValueError("vecnorm_update must be 'step' or 'rollout'")
        self.vecnorm_update = vecnorm_update
        self.f32 = False
        self.i8x4 = False
        self.blob = None
        self.attention = False
        self.attention_ln = False
        # SB3 VecFrameStack(n_stack) between the env and the policy
        # (code/lorenz_filter/train.py:115): the stack is carried on the device
        self.frame_stack = int(frame_stack)
        if self.frame_stack not in (1, 4):
            raise ValueError("frame_stack must be 1 or 4 (the fused kernel's instantiations)")
        if self.frame_stack > 1 and obs_rms is not None:
            raise ValueError("the frame-stacked rollout stacks raw observations (no VecNormalize)")
        self.last_stack = None
        self.last_obs = None
        self.last_episode_starts = torch.ones((self.n,), dtype=torch.float32, device=self.device)
        if state_dict is not None:
            self.set_params(state_dict)

    def set_params(self, state_dict):
        """Pack and upload the actor-critic weights (call after every optimizer step).
        A state_dict with code/train.py's AttentionFeaturesExtractor selects the
        attention kernel (lz_rollout_policy_attn), any other the MlpPolicy kernel."""
        self.attention = is_attention_policy(state_dict)
        self.attention_ln = is_attention_ln_policy(state_dict)
        if self.frame_stack > 1 and not self.attention_ln:
            raise ValueError("frame_stack > 1 runs code/lorenz_filter/train.py's policy "
                             "(the residual + LayerNorm attention extractor)")
        self.f32 = self.precision != "bf16"
        self.i8x4 = self.precision == "i8x4"
        if self.i8x4 and not (self.attention or self.attention_ln):
            if self.env.system_name not in ("lorenz3", "lorenz4", "pmsm", "hr"):
                raise ValueError("the i8x4 MlpPolicy runs LORENZ3 / LORENZ4 / PMSM / HR")
            if self.obs_rms is not None and self.training and self.vecnorm_update != "rollout":
                raise ValueError("precision='i8x4' with a training VecNormalize needs "
                                 "vecnorm_update='rollout' (the per-step collect is float32)")
        if self.attention_ln:
            if self.obs_rms is not None:
                raise ValueError("the LayerNorm attention rollout takes raw observations")
            blob = (pack_attn_ln_policy_i8x4 if self.i8x4 else
                    pack_attn_ln_policy_f32 if self.f32 else pack_attn_ln_policy)(
                state_dict, self.frame_stack * self.O, self.A)
        elif self.attention:
            blob = (pack_attn_policy_i8x4 if self.i8x4 else
                    pack_attn_policy_f32 if self.f32 else pack_attn_policy)(state_dict, self.O, self.A)
        else:
            blob = (pack_policy_i8x4 if self.i8x4 else
                    pack_policy_f32 if self.f32 else pack_policy)(state_dict, self.O, self.A)
        if self.vecnorm_update == "step" and (not self.f32 or self.attention or self.attention_ln):
            raise ValueError("vecnorm_update='step' runs the float32 MlpPolicy kernel")
        if self.f32:  # the packer's format tag against the launch this collector will make
            want = blob_format(self.attention, self.attention_ln, self.i8x4)
            got = int(nat.lib.lz_policy_blob_format(blob.ctypes.data, blob.size))
            if got != want:
                raise nat.LorenzEnvError(nat.LZ_ERR_INVALID, "policy blob format %d, the launch "
                                         "expects %d" % (got, want))
        self.blob = torch.from_numpy(blob).to(self.device)

    @property
    def per_step_vecnorm(self):
        """True when the collect updates obs_rms in SB3's per-step order."""
        return (self.obs_rms is not None and self.training and self.f32 and not self.attention
                and not self.attention_ln and self.vecnorm_update != "rollout")

    def _rms_update_obs(self, x):
        """VecNormalize.reset()'s obs_rms.update(obs) in the per-step kernel's moment order."""
        rms = self.obs_rms
        x = x.reshape(x.shape[0], self.O).contiguous()
        if self.group is None:
            nat.check(nat.lib.lz_rms_update_obs(rms._h, x.data_ptr(), x.shape[0], None))
            return
        mom = torch.empty((1 + 2 * self.O,), dtype=torch.float64, device=self.device)
        nat.check(nat.lib.lz_rms_update_obs(rms._h, x.data_ptr(), x.shape[0], mom.data_ptr()))
        dist.all_reduce(mom, group=self.group)
        nat.check(nat.lib.lz_rms_update(rms._h, ctypes.c_void_p(mom.data_ptr())))

    def reset(self):
        """VecEnv.reset(): fresh episodes; the next rollout starts from their obs."""
        obs = self.env.reset()
        self.last_obs = obs.clone()
        # StackedObservations.reset: zeros, the first frame last
        self.last_stack = torch.zeros((self.n, self.frame_stack * self.O), dtype=torch.float32,
                                      device=self.device)
        self.last_stack[:, -self.O:] = obs
        self.last_episode_starts.fill_(1.0)
        if self.obs_rms is not None and self.training:
            if self.per_step_vecnorm:
                self._rms_update_obs(self.last_obs)
            else:
                self.obs_rms.update(self.last_obs, self.group)
        return self.last_obs

    def collect(self, K):
        if self.blob is None:
            raise RuntimeError("set_params() first")
        if self.last_obs is None:
            self.reset()
        n, O, A, dev = self.n, self.O, self.A, self.device
        f32 = torch.float32
        SO = self.frame_stack * O if self.attention_ln else O
        obs_buf = torch.empty((K, n, SO), dtype=f32, device=dev)
        act_buf = torch.empty((K, n, A), dtype=f32, device=dev)
        logp = torch.empty((K, n), dtype=f32, device=dev)
        val = torch.empty((K, n), dtype=f32, device=dev)
        rew = torch.empty((K, n), dtype=f32, device=dev)
        done = torch.empty((K, n), dtype=torch.uint8, device=dev)
        last_val = torch.empty((n,), dtype=f32, device=dev)
        obs_last = torch.empty((n, O), dtype=f32, device=dev)
        per_step = self.per_step_vecnorm
        want_mom = self.obs_rms is not None and self.training and not per_step
        mom = torch.empty((1 + 2 * O,), dtype=torch.float64, device=dev) if want_mom else None
        didx = tobs = ndone = None
        if self.capture_terminal:
            didx = torch.empty((self.capture_terminal,), dtype=torch.int64, device=dev)
            tobs = torch.empty((self.capture_terminal, O), dtype=f32, device=dev)
            ndone = torch.zeros((1,), dtype=torch.int32, device=dev)
        r = nat.LzPolicyRolloutArgs()
        r.K = int(K)
        r.flags = ((nat.POLICY_DETERMINISTIC if self.deterministic else 0)
                   | (nat.POLICY_BOOTSTRAP if self.bootstrap else 0)
                   | (nat.POLICY_I8X4 if self.i8x4 else 0))
        r.blob, r.obs_in, r.obs_last = _p(self.blob), _p(self.last_obs), _p(obs_last)
        r.obs_norm = _p(self.obs_rms.state) if self.obs_rms is not None and not per_step else None
        r.norm_eps, r.clip_obs, r.gamma = self.norm_eps, self.clip_obs, self.gamma
        r.act_low, r.act_high = self.act_low, self.act_high
        r.obs_buf, r.act_buf, r.logp_buf, r.val_buf = _p(obs_buf), _p(act_buf), _p(logp), _p(val)
        r.rew_buf, r.done_buf, r.last_values = _p(rew), _p(done), _p(last_val)
        r.obs_moments = _p(mom)
        r.done_idx, r.terminal_obs, r.cap, r.n_done = _p(didx), _p(tobs), self.capture_terminal, _p(ndone)
        stack_out = None
        # the rollout runs on the env handle's stream; the caller's current stream (where
        # the buffers above were allocated and blob / last_obs written, and where the
        # follow-up kernels below run) is ordered around it both ways
        caller = torch.cuda.current_stream(dev)
        es = self.env.stream
        if es != caller:
            es.wait_stream(caller)
        if self.attention_ln:
            stack_out = torch.empty((n, SO), dtype=f32, device=dev)
            launch = (nat.lib.lz_rollout_policy_attn_stack_f32 if self.f32
                      else nat.lib.lz_rollout_policy_attn_stack)
            nat.check(launch(self.env._h, ctypes.byref(r), self.frame_stack, _p(self.last_stack),
                             _p(stack_out)))
        elif per_step:
            state = ctypes.c_void_p(self.obs_rms.state.data_ptr())
            if self.group is None:
                nat.check(nat.lib.lz_rollout_policy_f32_vn(self.env._h, ctypes.byref(r), state))
            else:  # every step's batch moments all-reduced before its update
                mom = torch.empty((1 + 2 * O,), dtype=torch.float64, device=dev)
                rh = self.obs_rms._h
                nat.check(nat.lib.lz_rms_set_stream(rh, ctypes.c_void_p(caller.cuda_stream)))
                for k in range(K + 1):
                    nat.check(nat.lib.lz_policy_step_f32(self.env._h, ctypes.byref(r), k, state,
                                                         ctypes.c_void_p(mom.data_ptr()) if k < K
                                                         else None))
                    if k < K:
                        if es != caller:
                            caller.wait_stream(es)
                        dist.all_reduce(mom, group=self.group)
                        nat.check(nat.lib.lz_rms_update(rh, ctypes.c_void_p(mom.data_ptr())))
                        if es != caller:
                            es.wait_stream(caller)
        else:
            launch = ((nat.lib.lz_rollout_policy_attn_f32 if self.f32 else nat.lib.lz_rollout_policy_attn)
                      if self.attention else
                      nat.lib.lz_rollout_policy_f32 if self.f32 else nat.lib.lz_rollout_policy)
            nat.check(launch(self.env._h, ctypes.byref(r)))
        if es != caller:
            caller.wait_stream(es)
        starts = torch.empty((K, n), dtype=f32, device=dev)
        carry = torch.empty((n,), dtype=f32, device=dev)
        nat.check(nat.lib.lz_episode_starts(n, K, _p(done), _p(self.last_episode_starts),
                                            _p(starts), _p(carry), dev.index,
                                            ctypes.c_void_p(caller.cuda_stream)))
        self.last_episode_starts = carry
        self._keep = (self.blob, self.last_obs, self.last_stack)  # alive until consumed
        self.last_obs = obs_last
        if stack_out is not None:
            self.last_stack = stack_out
        if want_mom:
            if self.group is not None:
                dist.all_reduce(mom, group=self.group)
            nat.check(nat.lib.lz_rms_update(self.obs_rms._h, ctypes.c_void_p(mom.data_ptr())))
        return RolloutBatch(obs_buf, act_buf, logp, val, rew, done, starts, last_val, obs_last,
                            mom, didx, tobs, ndone, stack_out)

    def compute_returns_and_advantage(self, batch):
        """RolloutBuffer.compute_returns_and_advantage(last_values, dones) on device."""
        K, n = batch.rewards.shape
        adv = torch.empty_like(batch.rewards)
        ret = torch.empty_like(batch.rewards)
        nat.check(nat.lib.lz_gae(n, K, _p(batch.rewards), _p(batch.values), _p(batch.dones),
                                 _p(batch.last_values), self.gamma, self.gae_lambda, _p(adv), _p(ret),
                                 self.device.index,
                                 ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)))
        batch.advantages, batch.returns = adv, ret
        return adv, ret
