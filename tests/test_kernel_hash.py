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
