"""Diagnostic: where a fused rollout and K single steps of the same batch part ways.
Usage: python tools/diag_rollout_steps.py <system> <n> [variant] [max_episode_steps]
Prints, for the first differing step, the differing env ids, both rows, and the done
history of those envs on both paths."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-lorenz_amd"))
import gym_lorenz as gl  # noqa: E402


def main():
    system, n = sys.argv[1], int(sys.argv[2])
    variant = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    mes = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    K = 33
    kw = {"add_noise": True} if system in ("pmsm", "hr") else {}
    a_be = gl.BatchedEnv(system, n, dtype="float32", seed=4, max_episode_steps=mes, variant=variant, **kw)
    b_be = gl.BatchedEnv(system, n, dtype="float32", seed=4, max_episode_steps=mes, **kw)
    a_be.reset()
    b_be.reset()
    A = torch.from_numpy(np.random.default_rng(3).uniform(-1.5, 1.5, (K, n, a_be.action_dim))
                         .astype(np.float32)).cuda()
    obs, rew, done, (didx, tobs, nd) = a_be.rollout(A, capture_terminal=K * n)
    obs, rew, done = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy()
    so, sr, sd = [], [], []
    for k in range(K):
        o, r, d = b_be.step(A[k])
        so.append(o.cpu().numpy().copy())
        sr.append(r.cpu().numpy().copy())
        sd.append(d.cpu().numpy().copy())
    so, sr, sd = np.stack(so), np.stack(sr), np.stack(sd)
    print("system %s n %d variant %d: rollout dones %d, step dones %d" %
          (system, n, variant, int((done != 0).sum()), int((sd != 0).sum())))
    for k in range(K):
        bo = obs[k].view(np.uint32) != so[k].view(np.uint32)
        bo &= ~(np.isnan(obs[k]) & np.isnan(so[k]))
        br = (rew[k].view(np.uint32) != sr[k].view(np.uint32)) & ~(np.isnan(rew[k]) & np.isnan(sr[k]))
        bd = done[k] != sd[k]
        envs = np.unique(np.concatenate([np.nonzero(bo.any(1))[0], np.nonzero(br)[0], np.nonzero(bd)[0]]))
        if len(envs):
            print("first differing step %d: %d envs, first ids %s" % (k, len(envs), envs[:16].tolist()))
            for e in envs[:4]:
                print(" env", e, "tile", e // 256, "lane", e % 256)
                print("  rollout obs", obs[k, e].tolist(), "rew", float(rew[k, e]), "done", int(done[k, e]))
                print("  step    obs", so[k, e].tolist(), "rew", float(sr[k, e]), "done", int(sd[k, e]))
                print("  rollout done history", done[:k + 1, e].tolist())
                print("  step    done history", sd[:k + 1, e].tolist())
                print("  rollout rew history", rew[:k + 1, e].tolist())
            return
    print("identical over %d steps" % K)


if __name__ == "__main__":
    main()
