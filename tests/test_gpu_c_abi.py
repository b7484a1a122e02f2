"""GPU: the C-ABI driven from plain C (tests/c_abi/abi_smoke.c, gcc + libamdhip64, no
Python in the loop) -- LORENZ3 lz_step and PMSM lz_rollout bit-exact vs the oracle."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_c_program_drives_the_abi(tmp_path):
    import oracle

    oracle.lib()  # builds liblz_oracle.so if needed
    gcc = shutil.which("gcc")
    assert gcc, "gcc is part of the image"
    lib_dir = os.path.join(ROOT, "gym-lorenz_amd", "gym_lorenz")
    orc_dir = os.path.join(ROOT, "oracle")
    exe = tmp_path / "abi_smoke"
    subprocess.check_call([
        gcc, "-O2", "-std=c11", "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
        "-D__HIP_PLATFORM_AMD__", os.path.join(ROOT, "tests", "c_abi", "abi_smoke.c"),
        "-L", lib_dir, "-L", orc_dir, "-L", "/opt/rocm/lib", "-l:libgym_lorenz_amd.so",
        "-l:liblz_oracle.so", "-lamdhip64", "-lm", "-Wl,-rpath," + lib_dir,
        "-Wl,-rpath," + orc_dir, "-Wl,-rpath,/opt/rocm/lib", "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    print(out.stdout, out.stderr)
    assert out.returncode == 0, out.stderr
    assert "bit-exact" in out.stdout
