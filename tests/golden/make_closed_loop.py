"""Generate tests/golden/pmsm_closed_loop.npz -- the f2 closed-loop golden.

Test infrastructure only.  Run in the build container (needs /root/reference):

    python tests/golden/make_closed_loop.py

What the reference holds, and how each piece is read WITHOUT executing anything
from the files:
  * the eight trained A2C policies `pmsm_a2c_alpha_{a:.2f}_clean_model`
    (code/lorenz_pmsm/train.py:150-176: SB3 2.7.1 MlpPolicy, pi/vf [128,128] Tanh,
    saved by model.save as a zip archive without the .zip suffix): the archive member
    `policy.pth` is a torch state_dict, loaded with torch.load(weights_only=True);
  * their frozen VecNormalize statistics `pmsm_a2c_alpha_{a:.2f}_clean_vecnorm.pkl`
    (train.py:177 env.save): a protocol-4 pickle.  It is NOT unpickled: the opcode
    stream is walked with pickletools.genops (a pure parser: nothing imported, no
    object constructed) and obs_rms.mean / obs_rms.var are taken from the raw
    little-endian f8 bytes of their ndarray BUILD payloads, count / clip_obs /
    epsilon from their BINFLOAT opcodes;
  * the traces `PMSM_Origin_Data.xlsx` written by code/lorenz_pmsm/test_evaluate.py:
    61-166 (sheets e1_Error / e2_Error / e3_Error, columns alpha=1/2 ... 1/10, 2000
    rows of state1[i] - state2[i] after each closed-loop step), parsed with zipfile +
    xml.etree (the values are float32 numbers printed with 16 significant digits:
    rounding the text to the nearest float32 recovers them, checked below).

The protocol the traces come from (test_evaluate.py:61-166), restated for the tests:
  fresh env per alpha (lambda/Adam at their ctor values), reset, then state1 :=
  [10,-10,15] f32, state2 := [0,0,0] f32 (:75-76,100-102); obs0 from the injected
  state (:105-111); 2000 x { action = clip(policy mean(normalize_obs(obs)), -1, 1)
  (SB3 predict(deterministic=True), :119); obs = env.step(action) normalised with
  the frozen statistics (training=False, :92) ; record state1 - state2 (:123-125) }.
  The 2000th step truncates (TimeLimit 2000, gym_lorenz/__init__.py:17-22), so
  DummyVecEnv auto-resets the env from its unseeded RNG before row 2000 is recorded:
  that row is a random reset state and is not reproducible -- rows 1..1999 are.

Also stored: `cpu_*` -- the same protocol run here with the REFERENCE PMSM env class
itself (lorenz_env_try_pmsm.py, imported with the make_golden.py stubs) and an fp32
torch restatement of SB3's deterministic MlpPolicy predict: per step the raw obs the
policy saw, the action, the states before / after, and state1 - state2.

FINDING (printed by this script): the xlsx is NOT reproducible from the
shipped models.  The xlsx was written 2026-02-28T22:37 (docProps/core.xml); all eight
`*_clean_model` archives were trained 2026-03-02 (their `data` start_time), i.e. they
overwrote the models the xlsx came from.  Row 1 of the xlsx fixes each column's first
action (the slave's x1/x2 move by 50 * a * dt from zero), and for 6 of 8 columns it is
not the first action the shipped policy computes from the same injected state.  What
the xlsx still pins is the env: its rows obey the PMSM Euler step (the action-free x3
channel of the slave reconstructed from consecutive rows reproduces within 4 ulp).
"""
import io
import os
import pickletools
import sys
import xml.etree.ElementTree as ET
import zipfile

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
# test_evaluate.py:72 -- the column order of the xlsx
ALPHA_FRACTIONS = [(1, 2), (1, 3), (1, 4), (1, 6), (1, 7), (1, 8), (1, 9), (1, 10)]
STEPS = 2000
SD_KEYS = [
    "mlp_extractor.policy_net.0.weight", "mlp_extractor.policy_net.0.bias",
    "mlp_extractor.policy_net.2.weight", "mlp_extractor.policy_net.2.bias",
    "mlp_extractor.value_net.0.weight", "mlp_extractor.value_net.0.bias",
    "mlp_extractor.value_net.2.weight", "mlp_extractor.value_net.2.bias",
    "action_net.weight", "action_net.bias", "value_net.weight", "value_net.bias",
    "log_std",
]


def read_policy(path):
    import torch
    with zipfile.ZipFile(path) as z:
        sd = torch.load(io.BytesIO(z.read("policy.pth")), weights_only=True,
                        map_location="cpu")
    return {k: sd[k].numpy().astype(np.float32) for k in SD_KEYS}


def read_vecnorm(path):
    """obs_rms.{mean,var,count}, clip_obs, epsilon from the opcode stream (no unpickling).

    The stream (SB3 VecNormalize.__getstate__ pickled by env.save) holds, in order,
    key 'obs_rms' ... key 'mean' <ndarray BUILD with SHORT_BINBYTES of 6 f8>, key 'var'
    <same>, key 'count' BINFLOAT; later the top-level keys 'clip_obs', 'epsilon' each
    followed by a BINFLOAT.
    """
    data = open(path, "rb").read()
    out, key, target, in_obs_rms = {}, None, None, False
    for op, arg, _pos in pickletools.genops(data):
        if op.name in ("SHORT_BINUNICODE", "BINUNICODE", "UNICODE"):
            if arg == "obs_rms":
                in_obs_rms = True
            elif arg == "ret_rms":
                in_obs_rms = False
            if in_obs_rms and arg in ("mean", "var"):
                target = arg        # the next 48-byte payload is this ndarray's data
            key = arg
        elif op.name in ("SHORT_BINBYTES", "BINBYTES") and target is not None:
            if len(arg) == 48:
                out[target] = np.frombuffer(arg, "<f8").copy()
                target = None
        elif op.name == "BINFLOAT":
            if key == "count" and in_obs_rms and "count" not in out:
                out["count"] = arg
            elif key in ("clip_obs", "epsilon") and key not in out:
                out[key] = arg
    for k in ("mean", "var", "count", "clip_obs", "epsilon"):
        assert k in out, (path, k)
    return out


def read_xlsx(path):
    """{sheet name: array [rows-1, cols]} with the header row separated."""
    ns = {"m": "http://schemas.openxmlformats.org/spreadsheetml/2006/main"}
    res = {}
    with zipfile.ZipFile(path) as z:
        wb = ET.fromstring(z.read("xl/workbook.xml"))
        sheets = [s.get("name") for s in wb.find("m:sheets", ns)]
        for i, name in enumerate(sheets):
            root = ET.fromstring(z.read("xl/worksheets/sheet%d.xml" % (i + 1)))
            rows = root.find("m:sheetData", ns)
            header, vals = None, []
            for r in rows:
                cells = []
                for c in r:
                    if c.get("t") == "inlineStr":
                        cells.append(c.find("m:is/m:t", ns).text)
                    else:
                        v = c.find("m:v", ns)
                        cells.append(float(v.text) if v is not None else np.nan)
                if header is None:
                    header = cells
                else:
                    vals.append(cells)
            res[name] = (header, np.array(vals, np.float64))
    return res


# ----------------------------------------------------------------- CPU closed loop
def sb3_normalize_obs(obs, st):
    """VecNormalize._normalize_obs + normalize_obs' float32 cast (SB3 2.7.1)."""
    return np.clip((obs - st["mean"]) / np.sqrt(st["var"] + st["epsilon"]),
                   -st["clip_obs"], st["clip_obs"]).astype(np.float32)


def torch_mean_action(sd, obs):
    """ActorCriticPolicy._predict(deterministic=True): action_net(policy_net(obs))."""
    import torch
    t = {k: torch.from_numpy(v) for k, v in sd.items()}
    x = torch.from_numpy(obs[None])
    h = torch.tanh(torch.nn.functional.linear(x, t[SD_KEYS[0]], t[SD_KEYS[1]]))
    h = torch.tanh(torch.nn.functional.linear(h, t[SD_KEYS[2]], t[SD_KEYS[3]]))
    mu = torch.nn.functional.linear(h, t["action_net.weight"], t["action_net.bias"])
    return np.clip(mu.numpy()[0], -1.0, 1.0)   # BasePolicy.predict clips to the Box


def cpu_closed_loop(mod, alpha, sd, st, steps=STEPS):
    env = mod.PMSM_Sync_Env(alpha=alpha, add_noise=False)
    env.reset(seed=0)
    env.state1 = np.array([10.0, -10.0, 15.0], np.float32)         # :75,101
    env.state2 = np.array([0.0, 0.0, 0.0], np.float32)             # :76,102
    raw = np.concatenate((env.state1 - env.state2,
                          env._get_derivatives(env.state1, [0, 0])
                          - env._get_derivatives(env.state2, [0, 0]))).astype(np.float32)
    obs = sb3_normalize_obs(raw, st)
    e = np.zeros((steps, 3), np.float32)
    acts = np.zeros((steps, 2), np.float32)
    raw_obs = np.zeros((steps, 6), np.float32)     # what the policy saw at step k (raw)
    s1 = np.zeros((steps + 1, 3), np.float32)     # states before step k (k = steps: after)
    s2 = np.zeros((steps + 1, 3), np.float32)
    for k in range(steps):
        raw_obs[k] = raw
        s1[k], s2[k] = env.state1, env.state2
        a = torch_mean_action(sd, obs)
        acts[k] = a
        o, _r, term, trunc, _ = env.step(a)
        e[k] = env.state1 - env.state2
        s1[k + 1], s2[k + 1] = env.state1, env.state2
        if term or trunc:
            break  # DummyVecEnv would reset here (row STEPS-1 only)
        raw = np.asarray(o, np.float32)
        obs = sb3_normalize_obs(raw, st)
    return e, acts, raw_obs, s1, s2


def main():
    sys.path.insert(0, OUT)
    import make_golden as mg
    mg._install_stubs()
    mod = mg._load("lorenz_env_try_pmsm.py", "ref_pmsm")

    xl = read_xlsx(os.path.join(REF, "PMSM_Origin_Data.xlsx"))
    arrays = {}
    alphas = []
    xlsx_e = np.zeros((len(ALPHA_FRACTIONS), STEPS, 3), np.float32)
    cpu_e = np.zeros_like(xlsx_e)
    cpu_a = np.zeros((len(ALPHA_FRACTIONS), STEPS, 2), np.float32)
    cpu_obs = np.zeros((len(ALPHA_FRACTIONS), STEPS, 6), np.float32)
    cpu_s1 = np.zeros((len(ALPHA_FRACTIONS), STEPS + 1, 3), np.float32)
    cpu_s2 = np.zeros_like(cpu_s1)
    for j, (num, den) in enumerate(ALPHA_FRACTIONS):
        alpha = num / den
        alphas.append(alpha)
        tag = "%.2f" % alpha                                  # test_evaluate.py:82-83
        sd = read_policy(os.path.join(REF, "pmsm_a2c_alpha_%s_clean_model" % tag))
        st = read_vecnorm(os.path.join(REF, "pmsm_a2c_alpha_%s_clean_vecnorm.pkl" % tag))
        for k in SD_KEYS:
            arrays["a%d/%s" % (j, k)] = sd[k]
        for k in ("mean", "var"):
            arrays["a%d/obs_rms.%s" % (j, k)] = st[k]
        arrays["a%d/obs_rms.count" % j] = np.float64(st["count"])
        arrays["a%d/clip_obs" % j] = np.float64(st["clip_obs"])
        arrays["a%d/epsilon" % j] = np.float64(st["epsilon"])
        col = "alpha=1/%d" % den
        for i in range(3):
            header, vals = xl["e%d_Error" % (i + 1)]
            c = header.index(col)
            v = vals[:, c]
            assert v.shape == (STEPS,)
            f = v.astype(np.float32)
            # the writer printed each f32 with 16 significant digits: nearest-f32 of the
            # text is the recorded value (it lies within 1e-15 relative of the text)
            assert np.all(np.abs(f.astype(np.float64) - v) <= 1e-15 * np.abs(v) + 1e-300)
            xlsx_e[j, :, i] = f
        with np.errstate(all="ignore"):
            cpu_e[j], cpu_a[j], cpu_obs[j], cpu_s1[j], cpu_s2[j] = cpu_closed_loop(mod, alpha, sd, st)
        d = np.abs(cpu_e[j, :STEPS - 1] - xlsx_e[j, :STEPS - 1])
        eq = np.all(cpu_e[j, :STEPS - 1] == xlsx_e[j, :STEPS - 1], axis=1)
        first = int(np.argmin(eq)) if not eq.all() else STEPS - 1
        print("alpha=1/%-2d  rows bit-equal %4d/1999 (first diff row %4d)  max|d| %.3e  "
              "rms e(last 1000) xlsx %.4e cpu %.4e" % (
                  den, eq.sum(), first, d.max(),
                  np.sqrt(np.mean(xlsx_e[j, 999:1999] ** 2)),
                  np.sqrt(np.mean(cpu_e[j, 999:1999] ** 2))))
    time_axis = xl["e1_Error"][1][:, 0]
    np.savez_compressed(os.path.join(OUT, "pmsm_closed_loop.npz"), alphas=np.array(alphas),
                        xlsx_e=xlsx_e, time=time_axis, cpu_e=cpu_e, cpu_actions=cpu_a,
                        cpu_raw_obs=cpu_obs, cpu_state1=cpu_s1, cpu_state2=cpu_s2,
                        init_state1=np.array([10.0, -10.0, 15.0], np.float32),
                        init_state2=np.zeros(3, np.float32), **arrays)
    print("wrote", os.path.join(OUT, "pmsm_closed_loop.npz"))


if __name__ == "__main__":
    main()
