"""tools/kernel_hash.py (no GPU): the code hash bench.py requires before it attaches a
committed PMC traffic figure to roofline.traffic -- found for the headline kernel in the
built library, stable across calls, distinct between kernels, None for a name that is
not in the library."""
import os
import sys

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import kernel_hash  # noqa: E402

HEAD = "_ZN2lz6k_stepINS_5SysL3IfEEfLi0EEEvNS_5KArgsE"
PMSM = "_ZN2lz6k_stepINS_7SysPMSMEfLi0EEEvNS_5KArgsE"


def test_code_objects_present():
    objs = list(kernel_hash.code_objects())
    assert objs and all(o[:4] == b"\x7fELF" for o in objs)


def test_hash_found_stable_distinct():
    a = kernel_hash.kernel_code_sha256(HEAD)
    assert a and len(a) == 64
    assert kernel_hash.kernel_code_sha256(HEAD) == a
    assert kernel_hash.kernel_code_sha256(PMSM) not in (None, a)
    assert kernel_hash.kernel_code_sha256("_Z_no_such_kernel") is None
    assert kernel_hash.kernel_code_sha256(HEAD, "/nonexistent.so") is None


def test_entry_offset_masked():
    """The masked hash ignores only the descriptor's code-entry offset: it differs from
    the whole-descriptor hash, and both are stable."""
    a, b = kernel_hash.kernel_code_sha256(HEAD), kernel_hash.kernel_code_sha256(HEAD, mask_entry=False)
    assert a and b and a != b
    assert kernel_hash.kernel_code_sha256(HEAD, mask_entry=False) == b


def test_bench_kernel_names_exist():
    """Every kernel bench.py names as a line's dominant kernel is in the built library
    (k_step_multi at the one-generation sizes, k_step elsewhere, the rollouts)."""
    import bench

    cases = [("lorenz3", "step", 1 << 20), ("pmsm", "step", 262144), ("pmsm", "step", 1 << 20),
             ("hr", "step", 1 << 20), ("hr", "step", 1 << 21), ("lorenz4", "step", 1 << 20),
             ("lorenz3", "rollout", 32768), ("lorenz3", "rollout", 65536),
             ("lorenz3", "rollout", 262144), ("pmsm", "rollout", 32768), ("pmsm", "rollout", 262144),
             ("lorenz4", "rollout", 32768), ("lorenz4", "rollout", 49152), ("lorenz4", "rollout", 65536)]
    names = set()
    for system, mode, n in cases:
        k = bench.kernel_name(system, mode, n, no_done=system == "lorenz3")
        assert kernel_hash.kernel_code_sha256(k) is not None, k
        names.add(k)
    assert "_ZN2lz12k_step_multiINS_5SysHRIfEEfLi4ELb0EEEvNS_5KArgsE" in names
    # PMSM rollouts: the lane-pair kernel at 2 < 32-env waves per CU <= 4, one-wave groups
    # around it, the 256-lane kernel from 131,072
    assert "k_rolloutINS_7SysPMSMEfLi64E" in bench.kernel_name("pmsm", "rollout", 16384)
    assert bench.kernel_name("pmsm", "rollout", 32768) == "_ZN2lz14k_rollout_pairINS_7SysPMSMEfLi7EEEvNS_5KArgsE"
    assert "k_rolloutINS_7SysPMSMEfLi64E" in bench.kernel_name("pmsm", "rollout", 32800)
    assert "k_rollout_pair" in bench.kernel_name("pmsm", "rollout", 262144, variant=1 << 27)
    assert "k_rolloutINS_7SysPMSMEfLi64E" in bench.kernel_name("pmsm", "rollout", 4097, variant=1 << 28)
    # LORENZ4 f32 rollouts: one-wave groups below 3/4 x 256 x CUs envs, 256 lanes from there
    assert "k_rolloutINS_5SysL4IfEEfLi64E" in bench.kernel_name("lorenz4", "rollout", 40960)
    assert "k_rolloutINS_5SysL4IfEEfLi256E" in bench.kernel_name("lorenz4", "rollout", 49152)
    # the split-lane force bits: 512 two lanes per env for any system, 256 one lane
    for system, n, v, want in (("hr", 32768, 512, "k_rollout_splitINS_5SysHR"),
                               ("pmsm", 4097, 512, "k_rollout_splitINS_7SysPMSM"),
                               ("lorenz3", 32768, 256, "k_rolloutINS_5SysL3IfEEfLi64E")):
        k = bench.kernel_name(system, "rollout", n, variant=v)
        assert want in k and kernel_hash.kernel_code_sha256(k) is not None, (system, v, k)
    assert bench.step_tiles("pmsm", 262144) == 1 and bench.step_tiles("hr", 1 << 20) == 4
    assert bench.step_tiles("hr", 1 << 21) == 1 and bench.step_tiles("lorenz3", 1 << 20) == 4
    assert bench.step_tiles("lorenz3", 131072) == 1 and bench.step_tiles("lorenz3", 1 << 21) == 1
    assert bench.step_tiles("lorenz3", 262144) == 1 and bench.step_tiles("lorenz3", 229376) == 1
    assert "k_step_multiINS_5SysL3IfEEfLi2E" in bench.kernel_name("lorenz3", "step", 262144, variant=32768)
    assert "k_stepINS_5SysL3" in bench.kernel_name("lorenz3", "step", 262144)
    assert bench.step_tiles("lorenz3", 1 << 20, f64=True) == 1
    assert bench.step_tiles("lorenz3", 786432) == 4 and bench.step_tiles("lorenz3", 851968) == 1
    assert bench.step_tiles("pmsm", 786432) == 4 and bench.step_tiles("pmsm", 917504) == 1
    assert bench.step_tiles("hr", 786432) == 1 and bench.step_tiles("pmsm", 1 << 20) == 4
    assert "k_step_multiINS_5SysL3IfEEfLi4E" in bench.kernel_name("lorenz3", "step", 1 << 20)
