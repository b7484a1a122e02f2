"""NumPy restatement of stable-baselines3's RolloutBuffer.compute_returns_and_advantage
-- TEST INFRASTRUCTURE ONLY.

Third-party dependency absent from /root/reference and from this image:
stable-baselines3 2.7.1 (pinned by the reference's saved models' system_info.txt:3;
used by code/lorenz_filter/train.py:123-127 PPO(gae_lambda=0.95) and
code/lorenz_pmsm/train.py:173-178 A2C).  This restates its published algorithm
(common/buffers.py RolloutBuffer.compute_returns_and_advantage) in the same NumPy
expression order and dtypes (float32 buffers, python-float gamma / gae_lambda), to check
lz_gae.  The reference's own files pin nothing at this boundary: parity unpinned beyond
this restatement.
"""
import numpy as np


def compute_returns_and_advantage(rewards, values, episode_starts, last_values, dones,
                                  gamma, gae_lambda):
    """rewards / values / episode_starts: float32 [K, N]; last_values float32 [N];
    dones: bool [N] (the last step's dones).  Returns (advantages, returns) float32."""
    K = rewards.shape[0]
    advantages = np.zeros_like(rewards, dtype=np.float32)
    last_values = np.asarray(last_values, np.float32).flatten()
    last_gae_lam = 0
    for step in reversed(range(K)):
        if step == K - 1:
            next_non_terminal = 1.0 - dones.astype(np.float32)
            next_values = last_values
        else:
            next_non_terminal = 1.0 - episode_starts[step + 1]
            next_values = values[step + 1]
        delta = rewards[step] + gamma * next_values * next_non_terminal - values[step]
        last_gae_lam = delta + gamma * gae_lambda * next_non_terminal * last_gae_lam
        advantages[step] = last_gae_lam
    returns = advantages + values
    return advantages, returns
