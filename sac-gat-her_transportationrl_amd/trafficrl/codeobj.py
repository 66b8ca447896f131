"""Per-kernel code identity of libtrafficrl.so.

Counter summaries under profiles/ (rocprofv3 --pmc) describe one kernel's
machine code.  Keying them to the whole shared library drops them whenever
any other kernel changes; keying them to the kernel's own code keeps them
exactly as long as they are valid.  `kernel_code_hash` reads the gfx950
code objects embedded in the library (the `.hip_fatbin` section: clang
offload bundles, one per translation unit), finds every kernel symbol whose
mangled name contains the given substring, and hashes its machine code
(the function's bytes in `.text`) together with its kernel descriptor (the
`<name>.kd` object: register counts, LDS size, launch properties).

Plain ELF parsing, no ROCm tools: the same function runs in bench.py on the
GPU box and in tools/pmc_summary.py where the counters are summarised.
"""
from __future__ import annotations

import hashlib
import struct
from typing import Dict, List, Optional, Tuple

_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
_TARGET = b"gfx950"


def _sections(elf: bytes) -> List[Tuple[str, int, int, int, int, int, int]]:
    """(name, type, addr, offset, size, link, entsize) of every section of an ELF64 image."""
    shoff = struct.unpack_from("<Q", elf, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    raw = []
    for i in range(shnum):
        name, typ, _flags, addr, off, size, link, _info, _align, entsize = struct.unpack_from(
            "<IIQQQQIIQQ", elf, shoff + i * shentsize)
        raw.append((name, typ, addr, off, size, link, entsize))
    stro = raw[shstrndx][3]
    out = []
    for name, typ, addr, off, size, link, entsize in raw:
        end = elf.index(b"\0", stro + name)
        out.append((elf[stro + name:end].decode(), typ, addr, off, size, link, entsize))
    return out


def _code_objects(lib: bytes) -> List[bytes]:
    """The gfx950 code objects of every offload bundle in the library."""
    secs = _sections(lib)
    fat = [s for s in secs if s[0] == ".hip_fatbin"]
    if not fat:
        return []
    _, _, _, off, size, _, _ = fat[0]
    blob = lib[off:off + size]
    out = []
    pos = blob.find(_MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tlen]
            p += 24 + tlen
            if triple.endswith(_TARGET) and esize:
                out.append(blob[pos + eoff:pos + eoff + esize])
        pos = blob.find(_MAGIC, pos + 32)
    return out


def _symbols(co: bytes) -> Dict[str, Tuple[int, int, int]]:
    """name -> (value, size, section index) of the defined symbols of a code object."""
    secs = _sections(co)
    out = {}
    for name, typ, _addr, off, size, link, entsize in secs:
        if typ not in (2, 11) or not entsize:   # SHT_SYMTAB, SHT_DYNSYM
            continue
        stro = secs[link][3]
        for k in range(size // entsize):
            st_name, _info, _other, shndx, value, ssize = struct.unpack_from("<IBBHQQ", co, off + k * entsize)
            if not st_name or shndx == 0:
                continue
            end = co.index(b"\0", stro + st_name)
            out[co[stro + st_name:end].decode()] = (value, ssize, shndx)
    return out


def _bytes_at(co: bytes, secs, value: int, size: int, shndx: int) -> bytes:
    _name, _typ, addr, off, _size, _link, _ent = secs[shndx]
    return co[off + value - addr:off + value - addr + size]


def kernel_code_hash(lib_path: str, substr: str) -> Optional[str]:
    """sha256[:16] over (name, code bytes, descriptor bytes) of every gfx950
    kernel whose mangled name contains `substr`, in name order; None when no
    kernel matches."""
    with open(lib_path, "rb") as fh:
        lib = fh.read()
    h = hashlib.sha256()
    found = 0
    for co in _code_objects(lib):
        secs = _sections(co)
        syms = _symbols(co)
        for name in sorted(syms):
            if substr not in name or name.endswith(".kd") or name + ".kd" not in syms:
                continue
            v, s, i = syms[name]
            kv, ks, ki = syms[name + ".kd"]
            h.update(name.encode())
            h.update(_bytes_at(co, secs, v, s, i))
            h.update(_bytes_at(co, secs, kv, ks, ki))
            found += 1
    return h.hexdigest()[:16] if found else None


def kernel_names(lib_path: str) -> List[str]:
    """Mangled names of every gfx950 kernel in the library."""
    with open(lib_path, "rb") as fh:
        lib = fh.read()
    names = []
    for co in _code_objects(lib):
        syms = _symbols(co)
        names += [n for n in syms if n + ".kd" in syms]
    return sorted(names)
