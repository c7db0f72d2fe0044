"""Identity of a kernel's machine code in the built library.

A measurement taken on one build (PMC traffic per launch, tools/pmc_traffic.py)
is replayed into a bench line only when the line's build runs the same
machine code.  This reads libslime_rs.so's offload bundles (clang offload
bundle format: one per translation unit, each with a gfx950 ELF code object),
finds the kernel's symbol in the code object's symbol table and hashes its
instruction bytes.  Edits elsewhere in the sources leave the id unchanged;
any change to the kernel's code changes it.  Pure Python, nothing spawned.
"""
from __future__ import annotations

import hashlib
import struct

BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _gfx_code_objects(blob: bytes, arch: str = "gfx950"):
    """Every code object for `arch` in the bundles embedded in blob."""
    pos = blob.find(BUNDLE_MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + 24)[0]
        off = pos + 32
        for _ in range(n):
            e_off, e_size, tlen = struct.unpack_from("<QQQ", blob, off)
            triple = blob[off + 24: off + 24 + tlen].decode(errors="replace")
            off += 24 + tlen
            if triple.endswith(arch):
                yield blob[pos + e_off: pos + e_off + e_size]
        pos = blob.find(BUNDLE_MAGIC, pos + len(BUNDLE_MAGIC))


def _symbols(elf: bytes):
    """(name, value, size, section bytes) of the FUNC symbols of an ELF64 code object."""
    if elf[:4] != b"\x7fELF":
        return
    shoff = struct.unpack_from("<Q", elf, 0x28)[0]
    shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    for s in secs:
        if s[1] != 2:  # SHT_SYMTAB
            continue
        strtab = secs[s[6]]
        for k in range(s[5] // 24):
            st_name, st_info, _, st_shndx, st_value, st_size = struct.unpack_from("<IBBHQQ", elf, s[4] + 24 * k)
            if st_info & 0xF != 2 or st_shndx == 0 or st_shndx >= len(secs):  # STT_FUNC, defined
                continue
            so = strtab[4] + st_name
            name = elf[so: elf.index(b"\0", so)].decode(errors="replace")
            sec = secs[st_shndx]
            start = sec[4] + (st_value - sec[3])  # file offset of the symbol in its section
            yield name, elf[start: start + st_size]


def kernel_code_id(lib_path: str, fragments: tuple[str, ...]) -> str | None:
    """sha256[:16] of the machine code of the one kernel whose mangled name
    contains every fragment (None if absent or ambiguous)."""
    blob = open(lib_path, "rb").read()
    hits = []
    for co in _gfx_code_objects(blob):
        for name, code in _symbols(co):
            if all(f in name for f in fragments) and code:
                hits.append(code)
    if len(hits) != 1:
        return None
    return hashlib.sha256(hits[0]).hexdigest()[:16]
