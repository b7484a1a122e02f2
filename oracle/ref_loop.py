"""Per-env NumPy restatement of the reference's dynamic.py env as SB3's DummyVecEnv
drives it -- TEST / BASELINE INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).

The reference steps its envs one Python object at a time: DummyVecEnv.step_wait
(stable-baselines3 2.7.1) calls env.step(action) per env and copies each returned
observation into a float32 buffer.  `LorenzRefEnv.step` restates
code/gym-lorenz/gym_lorenz/envs/dynamic.py:61-90 with the same kind of Python-level
NumPy work per call (np.clip of three action components, scalar float64 element
arithmetic on a length-3 state, a 6-element list observation minus a zero int array,
the reward as a generator sum of abs values, the time accumulator), so that its
throughput stands for the reference's own per-env step on the host.  The reference
itself cannot run on the GPU box (it is not shipped there).
"""
import numpy as np

SIGMA, RHO, BETA, DT = 10.0, 28.0, 8.0 / 3.0, 0.01  # dynamic.py:8-33, 73-75


class LorenzRefEnv:
    def __init__(self, x0):
        self.state1 = np.array(x0, dtype=np.float64)
        self.state2 = np.zeros(6, dtype=np.int64)
        self.t = 0.0

    def step(self, action):
        u1 = np.clip(action[0], -500.0, 500.0)
        u2 = np.clip(action[1], -500.0, 500.0)
        u3 = np.clip(action[2], -500.0, 500.0)
        s = self.state1
        dx = SIGMA * (s[1] - s[0])
        dy = RHO * s[0] - s[1] - s[0] * s[2]
        dz = s[0] * s[1] - BETA * s[2]
        s[0] = s[0] + dx * DT + u1
        s[1] = s[1] + dy * DT + u2
        s[2] = s[2] + dz * DT + u3
        dx = SIGMA * (s[1] - s[0])
        dy = RHO * s[0] - s[1] - s[0] * s[2]
        dz = s[0] * s[1] - BETA * s[2]
        obs = [s[0], s[1], s[2], dx, dy, dz] - self.state2
        reward = -sum(abs(v) for v in obs[0:3])
        self.t = self.t + DT
        return obs, reward, self.t == 10, {}


def dummy_vec_step(envs, actions, buf_obs, buf_rew):
    """DummyVecEnv.step_wait's per-env loop (no resets: done never fires here)."""
    for i, env in enumerate(envs):
        obs, rew, _, _ = env.step(actions[i])
        buf_obs[i] = obs
        buf_rew[i] = rew
