"""GPU: the optional learner collectives over RCCL itself (backend "nccl" on ROCm), not
gloo.  The box has one GPU and RCCL refuses two ranks on one device, so this is one
rank: it executes the RCCL code paths on the hardware -- communicator init on cuda:0,
gather / scatter / all-reduce of device tensors -- that the 8-GPU runs use, and checks
their results:
  * gather_to_rank0 / scatter_from_rank0 round-trip a ragged shard unchanged;
  * allreduce_moments equals the float64 moments of the batch;
  * LorenzVecNormalize(group=WORLD) (LZ_VN_DEFER: the fused step leaves its moments,
    RCCL all-reduces them, lz_vecnorm_apply updates) is bit-identical to the in-kernel
    update path over 12 steps.
Scaling across GPUs stays unmeasured here (the driver's 8-GPU runs)."""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, q):
    for p in (HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "gym-lorenz_amd")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        import gym_lorenz as gl
        from gym_lorenz.parallel import allreduce_moments, gather_to_rank0, scatter_from_rank0
        from gym_lorenz.vec_normalize import LorenzVecNormalize

        res = {"backend": dist.get_backend()}
        n = 10_007
        x = torch.randn((n, 6), device=dev, dtype=torch.float32)
        g = gather_to_rank0(x, n)
        res["gather"] = bool(torch.equal(g, x))
        s = scatter_from_rank0(x * 2, n, x)
        res["scatter"] = bool(torch.equal(s, x * 2))
        cnt, mean, var = allreduce_moments(x)
        xd = x.double()
        res["moments"] = (float(cnt) == n and bool(torch.allclose(mean, xd.mean(0), rtol=1e-12, atol=1e-15))
                          and bool(torch.allclose(var, xd.var(0, unbiased=False), rtol=1e-9, atol=1e-12)))
        acts = np.random.default_rng(0).uniform(-1, 1, (12, 20037, 2)).astype(np.float32)
        outs = []
        for group in (dist.group.WORLD, None):
            vn = LorenzVecNormalize(gl.make_vec("lorenz_pmsm-v0", 20037, seed=7, max_episode_steps=5),
                                    norm_obs=True, norm_reward=True, group=group)
            vn.reset()
            run = []
            for k in range(12):
                o, r, d, _ = vn.step(acts[k])
                run.append((o.copy(), r.copy(), d.copy()))
            run.append((vn.obs_rms.mean.copy(), vn.obs_rms.var.copy(), np.array([vn.obs_rms.count])))
            outs.append(run)
            vn.close()
        res["vecnorm_defer_bitexact"] = all(
            np.array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))
            for ra, rb in zip(*outs) for a, b in zip(ra, rb))
        q.put(("ok", res))
    except Exception as e:  # noqa: BLE001
        q.put(("err", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_rccl_single_rank_collectives():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    status, res = q.get(timeout=240)
    p.join(timeout=60)
    assert status == "ok", res
    print("RCCL single rank:", res)
    assert res["backend"] == "nccl"
    assert res["gather"] and res["scatter"] and res["moments"] and res["vecnorm_defer_bitexact"], res
