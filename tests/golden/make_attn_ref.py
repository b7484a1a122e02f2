"""Generate tests/golden/attn_ref.npz from the REFERENCE's own attention extractors.

Test infrastructure only (build container; /root/reference does not exist on the GPU
box).  It loads the two `AttentionFeaturesExtractor` classes exactly as the reference
defines them -- /root/reference/code/train.py:52-94 (fc1 + ReLU, 8 tokens x 16, 4-head
nn.MultiheadAttention, post_attention_fc 128 -> 64 + ReLU) and
/root/reference/code/lorenz_filter/train.py:55-103 (the same plus the residual and
LayerNorm(16)) -- by executing those files as modules with their absent third-party
imports stubbed in sys.modules (gymnasium, stable_baselines3 -- whose
BaseFeaturesExtractor is an nn.Module holding features_dim, as in SB3 2.7.1
common/torch_layers.py -- the reference's own gym_lorenz package and
lorenz_filter/env_utils, none of which contributes arithmetic to the forward), then
builds the SB3 ActorCriticPolicy shape around each extractor (share_features_extractor:
features_extractor -> mlp_extractor.policy_net / value_net = Linear(64,128) Tanh
Linear(128,128) Tanh -> action_net / value_net; code/train.py:101-106 net_arch
pi=[128,128] vf=[128,128]), seeds the weights and records, in torch float32 on the CPU:

  <v>/<state_dict key>  the policy's parameters (SB3 state_dict keys, features_extractor.*)
  <v>/x                 4,096 inputs  (plain: HR obs, 6 dims; ln: VecFrameStack(4) of
                        them, 24 dims -- code/lorenz_filter/train.py:115)
  <v>/features          the reference extractor's output [4096, 64]
  <v>/mean, <v>/value   action_net(pi(features)) [4096, 2], value_net(vf(features)) [4096]

with v = "plain" (code/train.py) and "ln" (code/lorenz_filter/train.py).  Only arrays
are stored; nothing from the reference's source.  Run:

  python tests/golden/make_attn_ref.py        (needs /root/reference)
"""
import importlib.util
import os
import sys
import types

sys.dont_write_bytecode = True  # never write .pyc into /root/reference
os.environ.setdefault("MPLBACKEND", "Agg")

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

REF = "/root/reference/code"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "attn_ref.npz")
N, A, SEED = 4096, 2, 20240


class _Box:
    def __init__(self, low=None, high=None, shape=None, dtype=np.float32):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), np.dtype(dtype)


class BaseFeaturesExtractor(nn.Module):
    """SB3 2.7.1 common/torch_layers.py BaseFeaturesExtractor: an nn.Module that keeps
    the observation space and features_dim (no parameters, no arithmetic)."""

    def __init__(self, observation_space, features_dim=0):
        super().__init__()
        assert features_dim > 0
        self._observation_space = observation_space
        self._features_dim = features_dim

    @property
    def features_dim(self):
        return self._features_dim


def _install_stubs():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        for k, v in attrs.items():
            setattr(m, k, v)
        sys.modules[name] = m
        return m

    spaces = mod("gymnasium.spaces", Box=_Box)
    mod("gymnasium", spaces=spaces, Env=object, make=None, register=lambda **kw: None)
    mod("gym_lorenz")  # the reference's env package: registration only, unused here
    mod("env_utils", make_env=None)  # lorenz_filter/env_utils.py (train.py:49)
    sb3 = mod("stable_baselines3", DDPG=object, A2C=object, SAC=object, PPO=object)
    common = mod("stable_baselines3.common")
    sb3.common = common
    mod("stable_baselines3.common.evaluation", evaluate_policy=None)
    mod("stable_baselines3.common.noise", NormalActionNoise=object)
    mod("stable_baselines3.common.torch_layers", BaseFeaturesExtractor=BaseFeaturesExtractor)
    mod("stable_baselines3.common.vec_env", SubprocVecEnv=object, DummyVecEnv=object,
        VecFrameStack=object)


def _load(path, name):
    spec = importlib.util.spec_from_file_location(name, path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


class _MlpExtractor(nn.Module):  # SB3 MlpExtractor(64, net_arch pi/vf [128,128], Tanh)
    def __init__(self, f=64, h=128):
        super().__init__()
        self.policy_net = nn.Sequential(nn.Linear(f, h), nn.Tanh(), nn.Linear(h, h), nn.Tanh())
        self.value_net = nn.Sequential(nn.Linear(f, h), nn.Tanh(), nn.Linear(h, h), nn.Tanh())


class Sb3AttnPolicy(nn.Module):
    """The SB3 ActorCriticPolicy layout around a features extractor (shared by pi / vf)."""

    def __init__(self, extractor, act_dim):
        super().__init__()
        self.features_extractor = extractor
        self.mlp_extractor = _MlpExtractor()
        self.action_net = nn.Linear(128, act_dim)
        self.value_net = nn.Linear(128, 1)
        self.log_std = nn.Parameter(torch.zeros(act_dim))

    def forward(self, x):
        f = self.features_extractor(x)
        return (f, self.action_net(self.mlp_extractor.policy_net(f)),
                self.value_net(self.mlp_extractor.value_net(f)).squeeze(-1))


def _inputs(in_dim, g):
    """HR-like observations ([e/50, clip(m/20)], lorenz_env_try.py:150-156) with a spread
    that exercises every ReLU / softmax regime: e/50 in ~[-3, 3], m/20 in [-1, 1]."""
    base = torch.empty(N, 6)
    base[:, :3] = torch.randn(N, 3, generator=g) * 1.2
    base[:, 3:] = torch.rand(N, 3, generator=g) * 2 - 1
    if in_dim == 6:
        return base
    frames = [base + 0.05 * torch.randn(N, 6, generator=g) * k for k in range(3, -1, -1)]
    x = torch.cat(frames, 1)
    x[: N // 16, :18] = 0.0  # VecFrameStack's zeros before a fresh episode's frame
    return x


def main():
    _install_stubs()
    plain = _load(os.path.join(REF, "train.py"), "ref_code_train")
    filt = _load(os.path.join(REF, "lorenz_filter", "train.py"), "ref_lorenz_filter_train")
    out = {"torch_version": np.array(torch.__version__)}
    for tag, module, in_dim in (("plain", plain, 6), ("ln", filt, 24)):
        torch.manual_seed(SEED + in_dim)
        ext = module.AttentionFeaturesExtractor(_Box(-np.inf, np.inf, (in_dim,)), features_dim=64)
        pol = Sb3AttnPolicy(ext, A)
        g = torch.Generator().manual_seed(SEED + 1 + in_dim)
        with torch.no_grad():  # weights spread enough that the softmax is far from uniform
            for p in pol.parameters():
                p.add_(torch.randn(p.shape, generator=g) * (0.15 if p.dim() > 1 else 0.1))
            ext.attention_layer.in_proj_weight.mul_(4.0)  # sharp softmax: real attention
        x = _inputs(in_dim, g)
        with torch.no_grad():
            f, m, v = pol(x)
        for k, t in pol.state_dict().items():
            out["%s/%s" % (tag, k)] = t.detach().numpy().astype(np.float32)
        out[tag + "/x"] = x.numpy().astype(np.float32)
        out[tag + "/features"] = f.numpy().astype(np.float32)
        out[tag + "/mean"] = m.numpy().astype(np.float32)
        out[tag + "/value"] = v.numpy().astype(np.float32)
        print(tag, {k: v.shape for k, v in pol.state_dict().items()})
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
