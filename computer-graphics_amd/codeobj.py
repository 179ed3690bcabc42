"""Identity of a kernel's machine code inside libcgamd.so (measurement tooling).

The bench's executed-work roofline scales rocprofv3 SQ counters collected on
one build of a kernel; those counters describe that machine code only.
kernel_sha256(name) hashes the gfx950 code of every kernel whose (mangled)
name carries `name` -- the function bytes plus its kernel descriptor (`.kd`:
register counts, scratch, LDS; its code-entry offset masked, see below) -- so a profile records what it measured and
the bench can refuse to scale a stale profile.

Layout walked here: the library's `.hip_fatbin` section holds one clang
offload bundle per translation unit ("__CLANG_OFFLOAD_BUNDLE__", u64 entry
count, then per entry u64 offset, u64 size, u64 triple length, triple); the
gfx950 entry is an AMDGPU ELF64 code object whose symbol table locates each
kernel (STT_FUNC) and descriptor (STT_OBJECT, `<symbol>.kd`).
"""
from __future__ import annotations

import hashlib
import os
import struct

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
DEFAULT_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libcgamd.so")


def _sections(elf: bytes):
    """[(name, type, addr, offset, size, link, entsize)] of an ELF64 little-endian image."""
    if elf[:4] != b"\x7fELF" or elf[4] != 2 or elf[5] != 1:
        raise ValueError("not an ELF64 little-endian image")
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    raw = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    stroff = raw[shstrndx][4]

    def name(off):
        end = elf.index(b"\0", stroff + off)
        return elf[stroff + off:end].decode()
    return [(name(s[0]), s[1], s[3], s[4], s[5], s[6], s[9]) for s in raw]


def _code_objects(lib: bytes):
    """The gfx950 code objects of every offload bundle in a host library image."""
    secs = [s for s in _sections(lib) if s[0] == ".hip_fatbin"]
    if not secs:
        raise ValueError("no .hip_fatbin section")
    _, _, _, off, size, _, _ = secs[0]
    fat = lib[off:off + size]
    out, pos = [], 0
    while True:
        b = fat.find(MAGIC, pos)
        if b < 0:
            break
        n, = struct.unpack_from("<Q", fat, b + len(MAGIC))
        q = b + len(MAGIC) + 8
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", fat, q)
            triple = fat[q + 24:q + 24 + tlen].decode(errors="replace")
            q += 24 + tlen
            if "gfx950" in triple and esize:
                out.append(fat[b + eoff:b + eoff + esize])
        pos = q
    return out


def _symbols(co: bytes):
    """{symbol name: bytes} for the functions and objects of a code object."""
    secs = _sections(co)
    out = {}
    for name, typ, _, off, size, link, ent in secs:
        if typ != 2:          # SHT_SYMTAB
            continue
        stroff = secs[link][3]
        for k in range(size // ent):
            st_name, st_info, _, st_shndx, st_value, st_size = struct.unpack_from("<IBBHQQ", co, off + k * ent)
            if st_info & 0xF not in (1, 2) or not st_size or st_shndx == 0 or st_shndx >= len(secs):
                continue
            end = co.index(b"\0", stroff + st_name)
            sym = co[stroff + st_name:end].decode()
            _, _, saddr, soff, _, _, _ = secs[st_shndx]
            start = soff + (st_value - saddr)
            out[sym] = co[start:start + st_size]
    return out


_CACHE: dict = {}


def kernel_symbols(lib_path: str = DEFAULT_LIB):
    """{symbol: bytes} over every gfx950 code object in the library (cached per path + mtime)."""
    key = (lib_path, os.path.getmtime(lib_path))
    if key not in _CACHE:
        with open(lib_path, "rb") as f:
            lib = f.read()
        syms = {}
        for co in _code_objects(lib):
            syms.update(_symbols(co))
        _CACHE.clear()
        _CACHE[key] = syms
    return _CACHE[key]


def kernel_sha256(name: str, lib_path: str = DEFAULT_LIB):
    """SHA-256 over the code and descriptors of every kernel whose mangled name contains the
    identifier `name` (all template instances), or None when the library has none."""
    ident = f"{len(name)}{name}"
    syms = kernel_symbols(lib_path)
    hit = sorted(s for s in syms if ident in s and (s.endswith(".kd") or s + ".kd" in syms))
    if not hit:
        return None
    h = hashlib.sha256()
    for s in hit:
        b = syms[s]
        if s.endswith(".kd") and len(b) >= 24:
            # kernel_code_entry_byte_offset (bytes 16-23) is the distance from the
            # descriptor to the code: layout, which moves whenever another kernel
            # of the same code object changes size, not this kernel's machine code
            b = b[:16] + bytes(8) + b[24:]
        h.update(s.encode() + b"\0")
        h.update(b)
    return h.hexdigest()


def kernel_names(lib_path: str = DEFAULT_LIB, prefixes=("rt_", "rast_", "jpeg_", "star_")):
    """The identifiers of the library's kernels (one per template family) whose name starts with
    one of `prefixes`, from the mangled names of their descriptors."""
    import re
    out = set()
    for s in kernel_symbols(lib_path):
        if not s.endswith(".kd"):
            continue
        pos = 0
        while True:                     # <length><identifier> runs of the mangled name
            m = re.compile(r"\d+").search(s, pos)
            if not m:
                break
            n = int(m.group(0))
            ident = s[m.end():m.end() + n]
            if ident.startswith(prefixes):
                out.add(ident)
                break
            pos = m.end() + (n if ident[:1].isalpha() or ident[:1] == "_" else 0)
    return sorted(out)


if __name__ == "__main__":
    import sys
    for k in sys.argv[1:] or ["rt_lattice_kernel", "rt_lattice_lights_kernel", "rt_big_primary_kernel"]:
        print(k, kernel_sha256(k))
