"""Per-env NumPy restatement of the reference's dynamic.py env as SB3's DummyVecEnv
drives it -- TEST / BASELINE INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).

The reference steps its envs one Python object at a time: DummyVecEnv.step_wait
(stable-baselines3 2.7.1) calls env.step(action) per env and copies each returned
observation into a float32 buffer.  `LorenzRefEnv.step` restates
code/gym-lorenz/gym_lorenz/envs/dynamic.py:61-90 with the SAME Python-level NumPy work
per call, so that its throughput is the reference's own per-env cost on the host:
  * three np.clip calls on the action components (:63-65);
  * the observation as list - int64 array FOUR times per call, as the reference does it:
    the stale `self.state = self._get_observation()` (:67), `self.state = self.state0 -
    self.state2` (:82), `now = self._get_observation()` (:83) and the returned
    `self._get_observation()` (:90);
  * scalar element arithmetic on the float64 state through instance attributes
    (self.u / self.i / self.o, :70-79), the 6-element state0 list (:80), the reward as a
    generator sum of abs values (:84), the float time accumulator and its == test
    (:85-89).
tests/test_oracle_golden.py::test_ref_loop_restatement_matches_reference_fixture pins it bit for bit against the
reference's own outputs (tests/golden/l3.npz).  The reference itself cannot run on the
GPU box (it is not shipped there).
"""
import numpy as np


class LorenzRefEnv:
    def __init__(self, x0):
        # dynamic.py:8-33 constants, :35-47 reset state (x0 injected)
        self.input_min, self.input_max = -500.0, 500.0
        self.u, self.i, self.o = 10, 28, 8 / 3
        self.u1 = self.u2 = self.u3 = 0
        self.state1 = np.array(x0, dtype=np.float64)
        s = self.state1
        self.state0 = [s[0], s[1], s[2], self.u * (s[1] - s[0]),
                       self.i * s[0] - s[1] - s[0] * s[2], s[0] * s[1] - self.o * s[2]]
        self.state2 = np.array([0, 0, 0, 0, 0, 0])
        self.state = None
        self.t = 0

    def _get_observation(self):
        return self.state0 - self.state2

    def step(self, action):
        self.u1 = np.clip(action[0], self.input_min, self.input_max)
        self.u2 = np.clip(action[1], self.input_min, self.input_max)
        self.u3 = np.clip(action[2], self.input_min, self.input_max)
        self.state = self._get_observation()            # :67 (overwritten below)
        s = self.state1
        f0 = self.u * (s[1] - s[0])
        f1 = self.i * s[0] - s[1] - s[0] * s[2]
        f2 = s[0] * s[1] - self.o * s[2]
        s[0] = s[0] + f0 * 0.01 + self.u1
        s[1] = s[1] + f1 * 0.01 + self.u2
        s[2] = s[2] + f2 * 0.01 + self.u3
        self.state1 = s
        f0 = self.u * (s[1] - s[0])
        f1 = self.i * s[0] - s[1] - s[0] * s[2]
        f2 = s[0] * s[1] - self.o * s[2]
        self.state0 = [s[0], s[1], s[2], f0, f1, f2]
        self.state = self.state0 - self.state2          # :82
        now = self._get_observation()                   # :83
        reward = -sum(abs(v) for v in now[0:3])         # :84
        self.t = self.t + 0.01
        done = self.t == 10
        return self._get_observation(), reward, done, {}  # :90


def dummy_vec_step(envs, actions, buf_obs, buf_rew):
    """DummyVecEnv.step_wait's per-env loop (no resets: done never fires here)."""
    for i, env in enumerate(envs):
        obs, rew, _, _ = env.step(actions[i])
        buf_obs[i] = obs
        buf_rew[i] = rew
