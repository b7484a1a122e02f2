"""The C-ABI library loads, exports every entry point include/lorenz_env.h declares,
has the header's struct layout, fills the reference constants and rejects bad
arguments with status codes (no GPU needed: no compute call is made)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "lorenz_env.h")


@pytest.fixture(scope="module")
def nat():
    from gym_lorenz import _native

    return _native


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\w[\w \*]*?\b(lz_\w+)\s*\(", src, flags=re.M)))


def test_every_declared_symbol_is_exported(nat):
    names = declared_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(nat.lib, n), n
    # and the python binding binds exactly the declared set
    assert sorted(nat.exported_symbols()) == names
    out = subprocess.run(["nm", "-D", "--defined-only", nat.LIB_PATH], capture_output=True,
                         text=True).stdout
    exported = set(re.findall(r" T (lz_\w+)", out))
    assert set(names) <= exported


def test_struct_layout_matches_header(nat, tmp_path):
    """Compile a probe against the public header with gcc: sizes and offsets must
    equal the ctypes mirror."""
    c = tmp_path / "probe.c"
    c.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "lorenz_env.h"\n'
        "int main(void){printf(\"%zu %zu %zu %zu %zu %zu %zu %zu %d %d %d\\n\", sizeof(lz_config),"
        " offsetof(lz_config, params), offsetof(lz_config, t_done_step),"
        " offsetof(lz_config, alpha), sizeof(lz_info), offsetof(lz_config, seed),"
        " offsetof(lz_config, reserved), offsetof(lz_config, integrator), LZ_INT_EULER, LZ_INT_RK4,"
        " LZ_ABI_VERSION);return 0;}\n")
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-I", os.path.dirname(HEADER), str(c), "-o", str(exe)])
    got = [int(v) for v in subprocess.check_output([str(exe)]).split()]
    C = nat.LzConfig
    want = [ctypes.sizeof(C), C.params.offset, C.t_done_step.offset, C.alpha.offset,
            ctypes.sizeof(nat.LzInfo), C.seed.offset, C.reserved.offset, C.integrator.offset,
            nat.INT_EULER, nat.INT_RK4, nat.ABI_VERSION]
    assert got == want


def test_vecnorm_struct_layout_matches_header(nat, tmp_path):
    c = tmp_path / "probe_vn.c"
    c.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "lorenz_env.h"\n'
        "int main(void){printf(\"%zu %zu %zu %zu %d %d %d %d\\n\", sizeof(lz_vecnorm),"
        " offsetof(lz_vecnorm, gamma), offsetof(lz_vecnorm, clip_reward),"
        " offsetof(lz_vecnorm, flags), LZ_VN_TRAINING, LZ_VN_NORM_OBS, LZ_VN_NORM_REWARD,"
        " LZ_VN_DEFER);return 0;}\n")
    exe = tmp_path / "probe_vn"
    subprocess.check_call(["gcc", "-I", os.path.dirname(HEADER), str(c), "-o", str(exe)])
    got = [int(v) for v in subprocess.check_output([str(exe)]).split()]
    V = nat.LzVecNorm
    assert got == [ctypes.sizeof(V), V.gamma.offset, V.clip_reward.offset, V.flags.offset,
                   nat.VN_TRAINING, nat.VN_NORM_OBS, nat.VN_NORM_REWARD, nat.VN_DEFER]


def test_config_init_reference_constants(nat, orc):
    for name, sysid in (("l3", nat.LORENZ3), ("l4", nat.LORENZ4), ("pmsm", nat.PMSM),
                        ("hr", nat.HR)):
        cfg = nat.config_init(sysid)
        want = orc.PARAMS[name]
        assert list(cfg.params)[: len(want)] == want, name
        assert cfg.dtype == nat.F32 and cfg.num_envs == 1 and cfg.t_done_step == -1
    assert nat.config_init(nat.PMSM).alpha == np.float32(0.5)


def test_abi_version_and_errors(nat):
    # 2: lz_get_state / lz_set_state gained (indices, count) and lz_config the integrator
    assert nat.lib.lz_abi_version() == 2 == nat.ABI_VERSION
    cfg = nat.LzConfig()
    assert nat.lib.lz_config_init(ctypes.byref(cfg), 99) == nat.LZ_ERR_INVALID
    assert b"unknown system" in nat.lib.lz_last_error()
    h = ctypes.c_void_p()
    cfg = nat.config_init(nat.PMSM)
    cfg.dtype = nat.F64
    assert nat.lib.lz_create(ctypes.byref(cfg), ctypes.byref(h)) == nat.LZ_ERR_UNSUPPORTED
    cfg = nat.config_init(nat.LORENZ3)
    cfg.num_envs = 0
    assert nat.lib.lz_create(ctypes.byref(cfg), ctypes.byref(h)) == nat.LZ_ERR_INVALID
    cfg = nat.config_init(nat.LORENZ3)
    cfg.max_episode_steps = -1
    assert nat.lib.lz_create(ctypes.byref(cfg), ctypes.byref(h)) == nat.LZ_ERR_INVALID
    # the integrator: Euler (the reference) by default, RK4 opt-in for LORENZ3 / LORENZ4
    assert nat.config_init(nat.LORENZ3).integrator == nat.INT_EULER
    cfg = nat.config_init(nat.LORENZ3)
    cfg.integrator = 7
    assert nat.lib.lz_create(ctypes.byref(cfg), ctypes.byref(h)) == nat.LZ_ERR_INVALID
    assert b"unknown integrator" in nat.lib.lz_last_error()
    cfg = nat.config_init(nat.PMSM)
    cfg.integrator = nat.INT_RK4
    assert nat.lib.lz_create(ctypes.byref(cfg), ctypes.byref(h)) == nat.LZ_ERR_UNSUPPORTED
    assert b"RK4" in nat.lib.lz_last_error()
    # NULL handles are rejected, never dereferenced
    assert nat.lib.lz_step(None, None, None, None, None, None, None, None, None) == nat.LZ_ERR_INVALID
    assert nat.lib.lz_reset(None, None, None, None) == nat.LZ_ERR_INVALID
    vn = nat.LzVecNorm()
    assert nat.lib.lz_step_vecnorm(None, ctypes.byref(vn), *([None] * 7)) == nat.LZ_ERR_INVALID
    assert nat.lib.lz_vecnorm_apply(None, ctypes.byref(vn), *([None] * 9)) == nat.LZ_ERR_INVALID
    assert nat.lib.lz_destroy(None) == nat.LZ_OK
    assert nat.lib.lz_plane_elem_size(None, 0) == 0


def test_no_gpu_fails_loudly(nat):
    """Without a HIP device the product path raises -- it never falls back to CPU."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    cfg = nat.config_init(nat.LORENZ3)
    h = ctypes.c_void_p()
    st = nat.lib.lz_create(ctypes.byref(cfg), ctypes.byref(h))
    assert st == nat.LZ_ERR_HIP and nat.lib.lz_last_error()
    import gym_lorenz

    with pytest.raises(nat.LorenzEnvError):
        gym_lorenz.BatchedEnv("lorenz3", 16)
    with pytest.raises(nat.LorenzEnvError):
        gym_lorenz.make("lorenz_dynamic-v0")


def test_product_never_imports_the_oracle():
    pkg = os.path.join(ROOT, "gym-lorenz_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                src = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in src and "liblz_oracle" not in src, f
                assert "from oracle" not in src, f


def _fresh(code):
    import subprocess
    import sys

    from conftest import PKG

    return subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, %r)\n" % PKG + code],
                          capture_output=True, text=True, timeout=600)


def test_one_hip_runtime_when_gym_lorenz_is_imported_first():
    """`import gym_lorenz` before `import torch`: exactly one libamdhip64 is mapped,
    torch's (the library's libamdhip64.so.7 binds to it)."""
    r = _fresh("import gym_lorenz, torch, os\n"
               "from gym_lorenz import _native as nat\n"
               "rt = nat.hip_runtimes()\n"
               "assert len(rt) == 1 and rt == nat.HIP_RUNTIME, rt\n"
               "assert os.path.dirname(rt[0]) == os.path.realpath(os.path.join("
               "os.path.dirname(torch.__file__), 'lib')), rt\n"
               "print('ok')\n")
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def test_two_hip_runtimes_fail_loudly():
    """/opt/rocm's libamdhip64 loaded before torch: torch brings its own copy, so the
    process would hold two runtimes; importing gym_lorenz raises ImportError naming them
    instead of running on torch's streams from the other runtime."""
    import glob

    rocm = sorted(glob.glob("/opt/rocm/lib/libamdhip64.so.*"))
    if not rocm:
        pytest.skip("no /opt/rocm libamdhip64")
    r = _fresh("import ctypes\nctypes.CDLL(%r)\n"
               "try:\n    import gym_lorenz\nexcept ImportError as e:\n"
               "    print('refused:', e)\nelse:\n    print('imported')\n" % rocm[0])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "refused:" in r.stdout and "2 HIP runtimes" in r.stdout, r.stdout
