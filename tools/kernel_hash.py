"""Code hash of one kernel inside the built library: sha256 over the kernel's gfx950
machine code and its kernel descriptor (<name>.kd: register counts, LDS size, launch
attributes; its kernel_code_entry_byte_offset field -- bytes 16-23, where the code sits
relative to the descriptor -- is zeroed, so adding an unrelated kernel to the same
source file does not change the hash of one whose code did not change), read from the
.so's clang offload bundles.  A PMC traffic figure measured
for a kernel stays valid exactly as long as this hash does -- bench.py attaches a
committed profiles/**/*pmc_summary.json's traffic only when the summary's recorded hash
equals the running library's (tools/pmc_summary.py and tools/pmc_sq_summary.py record
it).  Pure Python (struct): no ROCm tools needed.

  python tools/kernel_hash.py <kernel mangled name> [lib.so]
"""
import hashlib
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_SO = os.path.join(ROOT, "gym-lorenz_amd", "gym_lorenz", "libgym_lorenz_amd.so")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _sections(elf):
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    raw = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    stro = raw[shstrndx][4]
    out = []
    for name, typ, flags, addr, off, size, link, info, align, entsize in raw:
        nm = elf[stro + name:elf.index(b"\0", stro + name)].decode()
        out.append({"name": nm, "type": typ, "addr": addr, "off": off, "size": size,
                    "link": link, "entsize": entsize})
    return out


def code_objects(so_path=DEFAULT_SO, arch="gfx950"):
    """The ELF code objects for `arch` in every offload bundle of the library."""
    data = open(so_path, "rb").read()
    pos = data.find(MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", data, pos + 24)
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode(errors="replace")
            p += 24 + tlen
            if arch in triple and size:
                yield data[pos + off:pos + off + size]
        pos = data.find(MAGIC, pos + 24)


def _symbols(elf):
    secs = _sections(elf)
    for s in secs:
        if s["type"] not in (2, 11):  # SHT_SYMTAB, SHT_DYNSYM
            continue
        strtab = secs[s["link"]]["off"]
        for i in range(s["size"] // 24):
            name, info, other, shndx, value, size = struct.unpack_from("<IBBHQQ", elf, s["off"] + 24 * i)
            nm = elf[strtab + name:elf.index(b"\0", strtab + name)].decode(errors="replace")
            yield nm, shndx, value, size, secs


def _sym_bytes(elf, want):
    for nm, shndx, value, size, secs in _symbols(elf):
        if nm == want and 0 < shndx < len(secs) and size:
            sec = secs[shndx]
            start = sec["off"] + (value - sec["addr"])
            return elf[start:start + size]
    return None


def kernel_code_sha256(kernel, so_path=DEFAULT_SO, mask_entry=True):
    """sha256 hex of the kernel's code + descriptor, or None when it is not in the
    library (or the library is missing).  mask_entry=False: the round-3 first form
    (descriptor hashed whole), for checking summaries recorded with it."""
    try:
        for elf in code_objects(so_path):
            code = _sym_bytes(elf, kernel)
            if code is None:
                continue
            kd = bytearray(_sym_bytes(elf, kernel + ".kd") or b"")
            if mask_entry and len(kd) >= 24:
                kd[16:24] = bytes(8)  # kernel_code_entry_byte_offset: layout, not code
            kd = bytes(kd)
            return hashlib.sha256(code + b"|" + kd).hexdigest()
    except (OSError, struct.error, ValueError, IndexError):
        return None
    return None


if __name__ == "__main__":
    print(kernel_code_sha256(sys.argv[1], *(sys.argv[2:3] or [DEFAULT_SO])))
