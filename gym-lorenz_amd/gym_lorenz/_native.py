"""ctypes binding of libgym_lorenz_amd.so (include/lorenz_env.h).

The library is the only compute path: there is no CPU fallback.  If it is missing
(not built) importing this module raises; if no HIP device is visible, lz_create
fails with LZ_ERR_HIP / LZ_ERR_INVALID and LorenzEnvError is raised.
"""
import ctypes
import os

# torch first: its ROCm wheel brings its own libamdhip64 / libhsa-runtime64, and the
# process must end up with torch's HSA runtime shared by both HIP runtimes.  Loading
# this library before torch (i.e. `import gym_lorenz` before `import torch`) leaves
# /opt/rocm's HSA runtime in the process, under which this library's hipGetDeviceCount
# finds no device on the MI355X boxes (measured; tests/test_gpu_parity.py::
# test_import_order_gym_lorenz_first).
import torch  # noqa: F401

_HERE = os.path.dirname(os.path.abspath(__file__))
# LZ_LIB_AB: an alternative build of the same library, for A/B timing tools only
LIB_PATH = os.environ.get("LZ_LIB_AB") or os.path.join(_HERE, "libgym_lorenz_amd.so")

LZ_OK, LZ_ERR_INVALID, LZ_ERR_UNSUPPORTED, LZ_ERR_HIP, LZ_ERR_STATE, LZ_ERR_OOM = range(6)
LORENZ3, LORENZ4, PMSM, HR = range(4)
T1, T2, TP, SC = range(4, 8)  # legacy, unregistered variants
F32, F64 = 0, 1
INT_EULER, INT_RK4 = 0, 1  # lz_config.integrator
INTEGRATORS = {"euler": INT_EULER, "rk4": INT_RK4}
ABI_VERSION = 2  # include/lorenz_env.h LZ_ABI_VERSION this binding is written against
FLAG_AUTORESET, FLAG_ADD_NOISE, FLAG_EVAL_MODE, FLAG_ADD_FILTER = 1, 2, 4, 8
DONE_TERMINATED, DONE_TRUNCATED = 1, 2
MAX_PARAMS = 16

# state plane ids (lorenz_env.h)
L3_X, L3_Y, L3_Z, L3_STEP = 0, 1, 2, 3
L4_M1, L4_S1, L4_STEP = 0, 4, 8
PMSM_S1, PMSM_S2, PMSM_LAMBDA, PMSM_M, PMSM_V, PMSM_ADAM_STEP, PMSM_STEP = 0, 3, 6, 7, 8, 9, 10
HR_M, HR_S, HR_SIGMA, HR_FA, HR_STEP = 0, 3, 6, 7, 9
T1_X, T1_STEP = 0, 3
T2_M1, T2_S1, T2_STEP = 0, 4, 8
TP_M, TP_S, TP_STEP = 0, 3, 6
SC_X, SC_STEP = 0, 3


class LorenzEnvError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__("lorenz_env status %d: %s" % (status, msg))
        self.status = status


class LzIoSizes(ctypes.Structure):
    """lz_io_sizes: the bytes each caller buffer of lz_step / lz_rollout must cover."""
    _fields_ = [(f, ctypes.c_int64) for f in ("actions", "noise", "obs", "rew", "done", "done_idx",
                                              "terminal_obs", "n_done")]


class LzConfig(ctypes.Structure):
    _fields_ = [
        ("system", ctypes.c_int32),
        ("dtype", ctypes.c_int32),
        ("num_envs", ctypes.c_int64),
        ("global_env_offset", ctypes.c_int64),
        ("seed", ctypes.c_uint64),
        ("device", ctypes.c_int32),
        ("max_episode_steps", ctypes.c_int32),
        ("flags", ctypes.c_uint32),
        ("alpha", ctypes.c_float),
        ("params", ctypes.c_double * MAX_PARAMS),
        ("t_done_step", ctypes.c_int32),
        ("reserved", ctypes.c_int32 * 6),  # reserved[0]: kernel tuning variant (A/B)
        ("integrator", ctypes.c_int32),
    ]


class LzInfo(ctypes.Structure):
    _fields_ = [
        ("state_dim", ctypes.c_int32),
        ("action_dim", ctypes.c_int32),
        ("obs_dim", ctypes.c_int32),
        ("init_dim", ctypes.c_int32),
        ("n_planes", ctypes.c_int32),
        ("bytes_per_env_step", ctypes.c_int32),
        ("counts_steps", ctypes.c_int32),
        ("state_io_bytes", ctypes.c_int32),
    ]


POLICY_DETERMINISTIC, POLICY_BOOTSTRAP, POLICY_I8X4 = 1, 2, 4
# lz_policy_blob_format: the format tag every float32 / i8x4 packer writes (LZ_BLOB_*)
(BLOB_UNKNOWN, BLOB_MLP_F32, BLOB_MLP_I8X4, BLOB_ATTN_F32, BLOB_ATTN_I8X4, BLOB_ATTN_LN_F32,
 BLOB_ATTN_LN_I8X4) = range(7)
POLICY_HIDDEN = 128


class LzMlpPolicy(ctypes.Structure):
    _fields_ = [("obs_dim", ctypes.c_int32), ("act_dim", ctypes.c_int32)] + [
        (name, ctypes.c_void_p) for name in (
            "pi_w1", "pi_b1", "pi_w2", "pi_b2", "vf_w1", "vf_b1", "vf_w2", "vf_b2",
            "act_w", "act_b", "val_w", "val_b", "log_std")]


class LzAttnPolicy(ctypes.Structure):
    _fields_ = [("obs_dim", ctypes.c_int32), ("act_dim", ctypes.c_int32)] + [
        (name, ctypes.c_void_p) for name in (
            "fc1_w", "fc1_b", "in_proj_w", "in_proj_b", "out_proj_w", "out_proj_b", "post_w",
            "post_b", "pi_w1", "pi_b1", "pi_w2", "pi_b2", "vf_w1", "vf_b1", "vf_w2", "vf_b2",
            "act_w", "act_b", "val_w", "val_b", "log_std")]


class LzAttnLnPolicy(ctypes.Structure):
    _fields_ = [("attn", LzAttnPolicy), ("ln_w", ctypes.c_void_p), ("ln_b", ctypes.c_void_p)]


class LzPolicyRolloutArgs(ctypes.Structure):
    _fields_ = [
        ("K", ctypes.c_int32),
        ("flags", ctypes.c_uint32),
        ("blob", ctypes.c_void_p),
        ("obs_in", ctypes.c_void_p),
        ("obs_last", ctypes.c_void_p),
        ("obs_norm", ctypes.c_void_p),
        ("norm_eps", ctypes.c_double),
        ("clip_obs", ctypes.c_double),
        ("gamma", ctypes.c_double),
        ("act_low", ctypes.c_float),
        ("act_high", ctypes.c_float),
        ("obs_buf", ctypes.c_void_p),
        ("act_buf", ctypes.c_void_p),
        ("logp_buf", ctypes.c_void_p),
        ("val_buf", ctypes.c_void_p),
        ("rew_buf", ctypes.c_void_p),
        ("done_buf", ctypes.c_void_p),
        ("last_values", ctypes.c_void_p),
        ("obs_moments", ctypes.c_void_p),
        ("done_idx", ctypes.c_void_p),
        ("terminal_obs", ctypes.c_void_p),
        ("cap", ctypes.c_int64),
        ("n_done", ctypes.c_void_p),
    ]


class LzVecNorm(ctypes.Structure):
    _fields_ = [
        ("obs_rms", ctypes.c_void_p),
        ("ret_rms", ctypes.c_void_p),
        ("returns", ctypes.c_void_p),
        ("moments", ctypes.c_void_p),
        ("gamma", ctypes.c_double),
        ("epsilon", ctypes.c_double),
        ("clip_obs", ctypes.c_double),
        ("clip_reward", ctypes.c_double),
        ("flags", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
    ]


VN_TRAINING, VN_NORM_OBS, VN_NORM_REWARD, VN_DEFER = 1, 2, 4, 8


class LzLaunchShape(ctypes.Structure):
    _fields_ = [("kernel", ctypes.c_int32), ("envs_per_wave", ctypes.c_int32),
                ("waves", ctypes.c_int32), ("grid", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("groups", ctypes.c_int32)]


# lz_get_launch_shape calls / kernels / flags (lorenz_env.h)
(CALL_STEP, CALL_ROLLOUT, CALL_ROLLOUT_POLICY, CALL_ROLLOUT_POLICY_F32, CALL_POLICY_STEP_F32,
 CALL_ROLLOUT_POLICY_ATTN, CALL_ROLLOUT_POLICY_ATTN_STACK, CALL_ROLLOUT_POLICY_ATTN_F32,
 CALL_ROLLOUT_POLICY_ATTN_STACK_F32, CALL_STEP_NOISE) = range(10)
KERNELS = {1: "step", 2: "step_multi", 3: "rollout", 4: "rollout_wave", 5: "rollout_split",
           6: "policy", 7: "policy_pair", 8: "policy_pair_pipe", 9: "policy_split",
           10: "policy_step", 11: "policy_attn", 12: "policy_attn_f32", 13: "rollout_pair"}
SHAPE_NO_DONE, SHAPE_GRID_STRIDE = 1, 2

VP = ctypes.c_void_p
_SIGS = {
    "lz_config_init": (ctypes.c_int, [ctypes.POINTER(LzConfig), ctypes.c_int32]),
    "lz_create": (ctypes.c_int, [ctypes.POINTER(LzConfig), ctypes.POINTER(VP)]),
    "lz_destroy": (ctypes.c_int, [VP]),
    "lz_get_info": (ctypes.c_int, [VP, ctypes.POINTER(LzInfo)]),
    "lz_get_config": (ctypes.c_int, [VP, ctypes.POINTER(LzConfig)]),
    "lz_set_stream": (ctypes.c_int, [VP, VP]),
    "lz_set_seed": (ctypes.c_int, [VP, ctypes.c_uint64]),
    "lz_sync": (ctypes.c_int, [VP]),
    "lz_reset": (ctypes.c_int, [VP, VP, VP, VP]),
    "lz_step": (ctypes.c_int, [VP, VP, VP, VP, VP, VP, VP, VP, VP]),
    "lz_rollout": (ctypes.c_int, [VP, ctypes.c_int32, VP, VP, VP, VP, VP, VP, ctypes.c_int64, VP]),
    "lz_step_host": (ctypes.c_int, [VP, VP, VP, VP, VP, VP]),
    "lz_resident_step": (ctypes.c_int, [VP, VP, VP, VP, VP, VP]),
    "lz_resident_stop": (ctypes.c_int, [VP]),
    "lz_resident_read_state": (ctypes.c_int, [VP, ctypes.c_int32, VP]),
    "lz_get_state": (ctypes.c_int, [VP, ctypes.c_int32, VP, VP, ctypes.c_int64]),
    "lz_set_state": (ctypes.c_int, [VP, ctypes.c_int32, VP, VP, ctypes.c_int64]),
    "lz_plane_elem_size": (ctypes.c_int32, [VP, ctypes.c_int32]),
    "lz_rms_create": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_double,
                                     ctypes.POINTER(VP)]),
    "lz_rms_destroy": (ctypes.c_int, [VP]),
    "lz_rms_set_stream": (ctypes.c_int, [VP, VP]),
    "lz_rms_state": (ctypes.c_int, [VP, ctypes.POINTER(VP), ctypes.POINTER(VP),
                                    ctypes.POINTER(VP)]),
    "lz_rms_moments": (ctypes.c_int, [VP, VP, ctypes.c_int32, ctypes.c_int64, VP]),
    "lz_rms_update": (ctypes.c_int, [VP, VP]),
    "lz_rms_update_obs": (ctypes.c_int, [VP, VP, ctypes.c_int64, VP]),
    "lz_rms_normalize": (ctypes.c_int, [VP, VP, ctypes.c_int32, ctypes.c_int64, VP, ctypes.c_int32,
                                        ctypes.c_double, ctypes.c_double]),
    "lz_returns_update": (ctypes.c_int, [VP, VP, ctypes.c_int32, VP, ctypes.c_int64, ctypes.c_double,
                                         ctypes.c_int32, ctypes.c_int32, VP]),
    "lz_step_vecnorm": (ctypes.c_int, [VP, ctypes.POINTER(LzVecNorm), VP, VP, VP, VP, VP, VP, VP]),
    "lz_vecnorm_apply": (ctypes.c_int, [VP, ctypes.POINTER(LzVecNorm), VP, VP, VP, VP, VP, VP, VP,
                                        VP, VP]),
    "lz_policy_blob_bytes": (ctypes.c_int64, []),
    "lz_policy_pack": (ctypes.c_int, [ctypes.POINTER(LzMlpPolicy), VP, ctypes.c_int64]),
    "lz_policy_pack_hidden": (ctypes.c_int, [ctypes.POINTER(LzMlpPolicy), ctypes.c_int32, VP,
                                             ctypes.c_int64]),
    "lz_rollout_policy": (ctypes.c_int, [VP, ctypes.POINTER(LzPolicyRolloutArgs)]),
    "lz_policy_f32_blob_bytes": (ctypes.c_int64, []),
    "lz_policy_blob_format": (ctypes.c_int32, [VP, ctypes.c_int64]),
    "lz_io_sizes_for": (ctypes.c_int, [ctypes.POINTER(LzConfig), ctypes.c_int32, ctypes.c_int64,
                                       ctypes.POINTER(LzIoSizes)]),
    "lz_policy_pack_f32": (ctypes.c_int, [ctypes.POINTER(LzMlpPolicy), ctypes.c_int32, VP,
                                          ctypes.c_int64]),
    "lz_rollout_policy_f32": (ctypes.c_int, [VP, ctypes.POINTER(LzPolicyRolloutArgs)]),
    "lz_policy_step_f32": (ctypes.c_int, [VP, ctypes.POINTER(LzPolicyRolloutArgs), ctypes.c_int32, VP,
                                          VP]),
    "lz_rollout_policy_f32_vn": (ctypes.c_int, [VP, ctypes.POINTER(LzPolicyRolloutArgs), VP]),
    "lz_attn_policy_blob_bytes": (ctypes.c_int64, []),
    "lz_attn_policy_pack": (ctypes.c_int, [ctypes.POINTER(LzAttnPolicy), VP, ctypes.c_int64]),
    "lz_rollout_policy_attn": (ctypes.c_int, [VP, ctypes.POINTER(LzPolicyRolloutArgs)]),
    "lz_attn_ln_policy_blob_bytes": (ctypes.c_int64, []),
    "lz_attn_ln_policy_pack": (ctypes.c_int, [ctypes.POINTER(LzAttnLnPolicy), VP, ctypes.c_int64]),
    "lz_rollout_policy_attn_stack": (ctypes.c_int, [VP, ctypes.POINTER(LzPolicyRolloutArgs),
                                                    ctypes.c_int32, VP, VP]),
    "lz_attn_policy_f32_blob_bytes": (ctypes.c_int64, []),
    "lz_attn_policy_pack_f32": (ctypes.c_int, [ctypes.POINTER(LzAttnPolicy), VP, ctypes.c_int64]),
    "lz_attn_ln_policy_pack_f32": (ctypes.c_int, [ctypes.POINTER(LzAttnLnPolicy), VP, ctypes.c_int64]),
    "lz_attn_policy_pack_i8x4": (ctypes.c_int, [ctypes.POINTER(LzAttnPolicy), VP, ctypes.c_int64]),
    "lz_policy_pack_i8x4": (ctypes.c_int, [ctypes.POINTER(LzMlpPolicy), ctypes.c_int32, VP,
                                           ctypes.c_int64]),
    "lz_attn_ln_policy_pack_i8x4": (ctypes.c_int, [ctypes.POINTER(LzAttnLnPolicy), VP, ctypes.c_int64]),
    "lz_rollout_policy_attn_f32": (ctypes.c_int, [VP, ctypes.POINTER(LzPolicyRolloutArgs)]),
    "lz_rollout_policy_attn_stack_f32": (ctypes.c_int, [VP, ctypes.POINTER(LzPolicyRolloutArgs),
                                                        ctypes.c_int32, VP, VP]),
    "lz_gae": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, VP, VP, VP, VP, ctypes.c_double,
                              ctypes.c_double, VP, VP, ctypes.c_int32, VP]),
    "lz_episode_starts": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, VP, VP, VP, VP,
                                         ctypes.c_int32, VP]),
    "lz_frame_stack": (ctypes.c_int, [VP, VP, VP, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_int32, ctypes.c_int32, VP]),
    "lz_get_launch_shape": (ctypes.c_int, [VP, ctypes.c_int32, ctypes.POINTER(LzLaunchShape)]),
    "lz_last_error": (ctypes.c_char_p, []),
    "lz_abi_version": (ctypes.c_int32, []),
}

if not os.path.exists(LIB_PATH):
    raise ImportError(
        "gym_lorenz: native library %s is missing -- build it with "
        "`make -C gym-lorenz_amd` (or __graft_entry__.build()); there is no CPU fallback"
        % LIB_PATH)


def hip_runtimes():
    """Real paths of the libamdhip64 files mapped into this process."""
    paths = set()
    with open("/proc/self/maps") as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 6 and os.path.basename(parts[5]).startswith("libamdhip64"):
                paths.add(os.path.realpath(parts[5]))
    return sorted(paths)


lib = ctypes.CDLL(LIB_PATH)
# One HIP runtime per process: the library resolves libamdhip64.so.7 to whichever copy
# is loaded first (torch's, since torch is imported above).  If something loaded
# /opt/rocm's copy before torch, torch runs on its own runtime and this library on the
# other: the hipStream_t / device pointers torch hands over (lz_set_stream, every
# buffer) would belong to a different runtime.  Refuse that loudly.
HIP_RUNTIME = hip_runtimes()
if len(HIP_RUNTIME) != 1:
    raise ImportError(
        "gym_lorenz: %d HIP runtimes are mapped in this process (%s); torch and "
        "libgym_lorenz_amd.so must share one.  Import torch (or gym_lorenz) before "
        "anything that loads a libamdhip64 directly." % (len(HIP_RUNTIME), ", ".join(HIP_RUNTIME)))
if not os.environ.get("LZ_LIB_AB") and lib.lz_abi_version() != ABI_VERSION:
    raise ImportError("gym_lorenz: %s has ABI version %d, this binding expects %d -- rebuild it"
                      % (LIB_PATH, lib.lz_abi_version(), ABI_VERSION))
for _name, (_res, _args) in _SIGS.items():
    try:
        _f = getattr(lib, _name)
    except AttributeError:
        # an older build loaded on purpose by the A/B tooling (tools/ab_lib.py sets
        # LZ_LIB_AB) may predate an entry point; the product library has them all
        if os.environ.get("LZ_LIB_AB"):
            continue
        raise
    _f.restype = _res
    _f.argtypes = _args


# The same library through a second CDLL object whose functions carry no argtypes: the
# per-env drop-in classes' hot call (envs/_single.py) passes prebuilt ctypes arguments
# and skips the per-call argtypes conversion.  Not for general use.
lib_fast = ctypes.CDLL(LIB_PATH)


def check(status):
    if status != LZ_OK:
        raise LorenzEnvError(status, lib.lz_last_error().decode(errors="replace"))


def config_init(system):
    cfg = LzConfig()
    check(lib.lz_config_init(ctypes.byref(cfg), system))
    return cfg


def launch_shape(handle, call):
    """lz_get_launch_shape as a dict: kernel name, envs_per_wave, waves, grid, groups, flags."""
    sh = LzLaunchShape()
    check(lib.lz_get_launch_shape(handle, int(call), ctypes.byref(sh)))
    return {"kernel": KERNELS.get(sh.kernel, sh.kernel), "envs_per_wave": sh.envs_per_wave,
            "waves": sh.waves, "grid": sh.grid, "groups": sh.groups,
            "no_done": bool(sh.flags & SHAPE_NO_DONE), "grid_stride": bool(sh.flags & SHAPE_GRID_STRIDE)}


def exported_symbols():
    return list(_SIGS)
