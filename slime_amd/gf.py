"""Python mirror of slime's ``internal/rs/gf`` Go API over the MI355X C-ABI.

MaxVal, MInverse and Raise are host scalars.  MapToGF / MapToGFWith /
MapFromGF take and return host memory, so their byte<->symbol codec runs on
the host cores where the bytes are (host_codec.cpp; slime_gf_codec_placement
can send it through the GPU codec kernels instead, gf_codec.hip).
Reference: /root/reference/internal/rs/gf/{gf,map}.go.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N

lib = N.lib

MaxVal = 4294967291  # map.go:7  (1<<32 - 5)


def MInverse(v: int) -> int:
    """gf.go:5 — v^(p-2) mod p."""
    return int(lib.slime_gf_minverse(v & 0xFFFFFFFF))


def Raise(x: int, n: int) -> int:
    """gf.go:46 — x^n mod p, Raise(x, 0) = 1."""
    return int(lib.slime_gf_raise(x & 0xFFFFFFFF, n & 0xFFFFFFFF))


def _bytes(b) -> np.ndarray:
    """A uint8 view of b (bytes, bytearray, memoryview, ndarray) without
    copying it; other byte sequences (e.g. a list of ints) go through bytes()."""
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b).view(np.uint8).reshape(-1)
    try:
        mv = memoryview(b).cast("B")
    except TypeError:
        mv = memoryview(bytes(b))
    return np.frombuffer(mv, dtype=np.uint8) if mv.nbytes else np.zeros(0, dtype=np.uint8)


def MapToGF(data) -> tuple[int, np.ndarray]:
    """map.go:15 — (mapping, symbols); mapping 0, else 1<<31, else a random fitting value."""
    src = _bytes(data)
    out = np.empty((src.size + 3) // 4, dtype=np.uint32)  # every word is written
    m = ctypes.c_uint32(0)
    N.check(lib.slime_gf_map_to_gf(src.ctypes.data if src.size else None, src.size, ctypes.byref(m),
                                   out.ctypes.data if out.size else None))
    return int(m.value), out


def MapToGFWith(data, n: int) -> np.ndarray:
    """map.go:74 — big-endian symbols XOR n."""
    src = _bytes(data)
    out = np.empty((src.size + 3) // 4, dtype=np.uint32)  # every word is written
    N.check(lib.slime_gf_map_to_gf_with(src.ctypes.data if src.size else None, src.size, n & 0xFFFFFFFF,
                                        out.ctypes.data if out.size else None))
    return out


_new_bytearray = ctypes.pythonapi.PyByteArray_FromStringAndSize
_new_bytearray.restype = ctypes.py_object
_new_bytearray.argtypes = [ctypes.c_char_p, ctypes.c_ssize_t]


def MapFromGF(n: int, v) -> bytearray:
    """map.go:103 — symbols XOR n as big-endian bytes (length 4*len(v)).

    Returns a bytearray: Go's []byte is mutable (and, like a bytearray, not
    usable as a map key), and the library writes the result in place with no
    extra 4*len(v)-byte copy.  The bytearray is created uninitialised (every
    byte is written by the codec), so its pages are first touched by the
    codec's threads, not by a zero-fill.  Use bytes(...) where an immutable,
    hashable value is needed."""
    words = np.ascontiguousarray(v, dtype=np.uint32)
    out = _new_bytearray(None, words.size * 4)
    ptr = (ctypes.c_char * len(out)).from_buffer(out) if out else None
    N.check(lib.slime_gf_map_from_gf(n & 0xFFFFFFFF, words.ctypes.data if words.size else None, words.size,
                                     ctypes.addressof(ptr) if ptr is not None else None))
    return out


def codec_placement(mode: int | None = None) -> int:
    """Where the three codec calls above run: 0 host cores (default), 1 GPU
    codec kernels; None queries.  Returns the placement in force before the call."""
    prev = int(lib.slime_gf_codec_placement(-1))
    if mode is not None:
        N.check(lib.slime_gf_codec_placement(int(mode)))
    return prev


def Seed(seed: int) -> None:
    """Seed MapToGF's random-fallback candidate stream (reference: rand.Uint32())."""
    lib.slime_gf_seed(seed & 0xFFFFFFFFFFFFFFFF)
