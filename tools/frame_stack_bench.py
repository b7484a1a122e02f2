"""lz_frame_stack throughput (VecFrameStack(4) of HR, code/lorenz_filter/train.py:115) at
1M envs: HIP-event time per call and algorithmic bytes (stack read + written, obs read,
done byte) against the 8 TB/s HBM roofline.  LZ_FRAME_STACK_ROWS=1 selects the per-row
kernel (A/B).  Prints one JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-lorenz_amd"))
import torch  # noqa: E402

from gym_lorenz import _native as nat  # noqa: E402

n, S, O = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20, 4, 6
st = torch.zeros((n, S * O), device="cuda")
obs = torch.randn((8, n, O), device="cuda")
done = (torch.rand((8, n), device="cuda") < 0.01).to(torch.uint8)
sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
for k in range(20):
    nat.check(nat.lib.lz_frame_stack(P(st), P(obs[k % 8]), P(done[k % 8]), n, S, O, 0, 0, sp))
torch.cuda.synchronize()
reps = 400
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for k in range(reps):
    nat.check(nat.lib.lz_frame_stack(P(st), P(obs[k % 8]), P(done[k % 8]), n, S, O, 0, 0, sp))
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / reps
b = 2 * S * O * 4 + O * 4 + 1
print(json.dumps({"kernel": "per-row" if os.environ.get("LZ_FRAME_STACK_ROWS") else "lds-tile",
                  "envs": n, "n_stack": S, "obs_dim": O, "us_per_call": us,
                  "bytes_per_env": b, "GBps": b * n / us / 1e3,
                  "frac_of_8TBps": b * n / us / 1e3 / 8000.0}))
