"""NumPy restatement of stable-baselines3's VecNormalize -- TEST INFRASTRUCTURE ONLY.

Third-party dependency absent from /root/reference and from this image:
stable-baselines3 2.7.1 (pinned by the reference's saved models' system_info.txt:3
and code/lorenz_pmsm/train.py's use of VecNormalize at :118,170).  This restates its
published algorithm (stable_baselines3/common/running_mean_std.py RunningMeanStd and
common/vec_env/vec_normalize.py VecNormalize.reset / step_wait / _update_reward /
normalize_obs / normalize_reward) in the same NumPy expression order and dtypes, to
check gym_lorenz.vec_normalize.LorenzVecNormalize.  The reference's own files pin
nothing at this boundary: parity unpinned beyond this restatement.
"""
import numpy as np


class RunningMeanStd:
    """SB3 RunningMeanStd(epsilon=1e-4, shape)."""

    def __init__(self, epsilon=1e-4, shape=()):
        self.mean = np.zeros(shape, np.float64)
        self.var = np.ones(shape, np.float64)
        self.count = epsilon

    def update(self, arr):
        batch_mean = np.mean(arr, axis=0)
        batch_var = np.var(arr, axis=0)
        batch_count = arr.shape[0]
        self.update_from_moments(batch_mean, batch_var, batch_count)

    def update_from_moments(self, batch_mean, batch_var, batch_count):
        delta = batch_mean - self.mean
        tot_count = self.count + batch_count
        new_mean = self.mean + delta * batch_count / tot_count
        m_a = self.var * self.count
        m_b = batch_var * batch_count
        m_2 = m_a + m_b + np.square(delta) * self.count * batch_count / tot_count
        new_var = m_2 / tot_count
        self.mean = new_mean
        self.var = new_var
        self.count = tot_count


class VecNormalizeRef:
    """VecNormalize arithmetic over (obs, rewards, dones, terminal obs) arrays."""

    def __init__(self, num_envs, obs_dim, training=True, norm_obs=True, norm_reward=True,
                 clip_obs=10.0, clip_reward=10.0, gamma=0.99, epsilon=1e-8):
        self.obs_rms = RunningMeanStd(shape=(obs_dim,))
        self.ret_rms = RunningMeanStd(shape=())
        self.clip_obs, self.clip_reward = clip_obs, clip_reward
        self.gamma, self.epsilon = gamma, epsilon
        self.training, self.norm_obs, self.norm_reward = training, norm_obs, norm_reward
        self.returns = np.zeros(num_envs)

    def normalize_obs(self, obs):
        if not self.norm_obs:
            return obs
        return np.clip((obs - self.obs_rms.mean) / np.sqrt(self.obs_rms.var + self.epsilon),
                       -self.clip_obs, self.clip_obs)

    def normalize_reward(self, reward):
        if self.norm_reward:
            reward = np.clip(reward / np.sqrt(self.ret_rms.var + self.epsilon), -self.clip_reward,
                             self.clip_reward)
        return reward

    def reset(self, obs):
        self.returns = np.zeros(len(self.returns))
        if self.training and self.norm_obs:
            self.obs_rms.update(obs)
        return self.normalize_obs(obs)

    def step(self, obs, rewards, dones, terminal_obs=None):
        """terminal_obs: {env index: raw terminal observation} for done envs."""
        if self.training and self.norm_obs:
            self.obs_rms.update(obs)
        obs = self.normalize_obs(obs)
        if self.training:
            self.returns = self.returns * self.gamma + rewards
            self.ret_rms.update(self.returns)
        rewards = self.normalize_reward(rewards)
        tn = {i: self.normalize_obs(o) for i, o in (terminal_obs or {}).items()}
        self.returns[dones] = 0
        return obs, rewards, dones, tn
