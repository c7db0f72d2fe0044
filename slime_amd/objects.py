"""Object-level data paths of slime's multi store over the MI355X C-ABI.

``write_chunks`` is the data path of ``Multi.writeChunks``
(internal/store/multi/multi_store.go:526-531, :554): MapToGF, splitVector,
one CreateParity per parity row, MapFromGF per part.  ``reconstruct`` is the
slow path of ``Multi.reconstruct`` (multi_store.go:215-241): MapToGFWith per
surviving chunk, RecoverData, MapFromGF, truncation to the object size.  Both
run on the GPU in one fused pass.  ``write_chunks_digest`` adds the chunks'
SHA-256 (store.DataV, store.go:104-110) and chunk-file FNV-1a headers
(storedir/directory.go:548-553), hashed on host threads while the device
pipeline runs; ``reconstruct_verify`` checks the object's SHA-256
(multi_store.go:244-249).  Storage and metadata stay with the caller.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np

from . import _native as N

lib = N.lib


def chunk_size(size: int, need: int) -> int:
    """Bytes per chunk: 4 * ceil(ceil(size/4) / need) (splitVector, multi_store.go:271-278)."""
    return int(lib.slime_rs_chunk_size(size, need))


def split_vector(data: np.ndarray, count: int) -> list[np.ndarray]:
    """The caller's splitVector (multi_store.go:271-299), for callers that keep
    the reference's call-by-call path: `count` parts of ceil(len/count)
    symbols, views into `data` where whole, a zero-padded copy for the short
    tail part and any empty trailing parts."""
    per = -(-data.size // count)
    parts = []
    for i in range(count):
        p = data[i * per:(i + 1) * per]
        if p.size != per:
            q = np.zeros(per, dtype=np.uint32)
            q[:p.size] = p
            p = q
        parts.append(p)
    return parts


def _bytes_view(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    return np.frombuffer(memoryview(data), dtype=np.uint8)


def write_chunks(data, need: int, total: int, out: Sequence[np.ndarray] | None = None, alias: bool = False,
                 device: int | None = None) -> tuple[int, list[np.ndarray]]:
    """(MappingValue, [total chunk byte arrays]) for an object, as writeChunks
    stores them.  `out`: caller-owned uint8 chunk buffers (>= chunk_size bytes
    each) written in place and returned as views.  alias=True returns the data
    chunks that lie wholly inside the object as views of `data` (no copy).
    `device`: run on that GPU (default: the thread's selection, else the
    library's device pool)."""
    buf = _bytes_view(data)
    chunks = _chunk_out(buf, need, total, out, alias)
    ptrs = (ctypes.c_void_p * max(len(chunks), 1))(*[c.ctypes.data for c in chunks])
    m = ctypes.c_uint32(0)
    with N.on_device(device):
        N.check(lib.slime_rs_write_chunks(buf.ctypes.data if buf.size else None, buf.size, need, total, ptrs,
                                          ctypes.byref(m)))
    return int(m.value), chunks


def _chunk_out(buf: np.ndarray, need: int, total: int, out, alias: bool = False) -> list[np.ndarray]:
    cb = chunk_size(buf.size, need) if need > 0 else 0
    if out is None:
        chunks = [np.empty(cb, dtype=np.uint8) for _ in range(max(total, 0))]
    else:
        if len(out) != total or any(o.dtype != np.uint8 or not o.flags.c_contiguous or not o.flags.writeable
                                    or o.size < cb for o in out):
            raise ValueError("write_chunks: out must be `total` writeable contiguous uint8 arrays of chunk_size bytes")
        chunks = [o[:cb] for o in out]
    if alias and cb:
        # Zero-copy data chunks: chunk j is the object's own bytes where it lies
        # wholly inside the object (views of `data`; slime_rs_write_chunks).
        for j in range(min(need, total)):
            if (j + 1) * cb <= buf.size:
                chunks[j] = buf[j * cb:(j + 1) * cb]
    return chunks


def write_chunks_digest(data, need: int, total: int, out: Sequence[np.ndarray] | None = None,
                        headers: bool = False, alias: bool = False, device: int | None = None
                        ) -> tuple[int, list[np.ndarray], list[bytes], list[bytes] | None]:
    """write_chunks plus each chunk's SHA-256 (what writeChunks' store.DataV
    stores, multi_store.go:554-556) and, with headers=True, each chunk file's
    8-byte FNV-1a-64 header over SHA-256 ‖ chunk (directory.go:548-553).
    Returns (mapping, chunks, shas, headers or None)."""
    buf = _bytes_view(data)
    chunks = _chunk_out(buf, need, total, out, alias)
    ptrs = (ctypes.c_void_p * max(len(chunks), 1))(*[c.ctypes.data for c in chunks])
    sha = np.zeros(max(total, 1) * 32, dtype=np.uint8)
    hdr = np.zeros(max(total, 1) * 8, dtype=np.uint8) if headers else None
    m = ctypes.c_uint32(0)
    with N.on_device(device):
        N.check(lib.slime_rs_write_chunks_digest(buf.ctypes.data if buf.size else None, buf.size, need, total, ptrs,
                                                 ctypes.byref(m), sha.ctypes.data,
                                                 hdr.ctypes.data if hdr is not None else None))
    shas = [sha[32 * i:32 * i + 32].tobytes() for i in range(max(total, 0))]
    hdrs = [hdr[8 * i:8 * i + 8].tobytes() for i in range(max(total, 0))] if hdr is not None else None
    return int(m.value), chunks, shas, hdrs


def sha256(data) -> bytes:
    """SHA-256 of a bytes-like object or array (sha256.Sum256)."""
    buf = _bytes_view(data)
    out = np.zeros(32, dtype=np.uint8)
    N.check(lib.slime_rs_sha256(buf.ctypes.data if buf.size else None, buf.size, out.ctypes.data))
    return out.tobytes()


def chunk_digests(chunks: Sequence, headers: bool = False) -> tuple[list[bytes], list[bytes] | None]:
    """SHA-256 of every chunk and, with headers=True, its chunk-file FNV-1a-64
    header (big-endian), hashed in parallel on the digest threads."""
    arrs = [_bytes_view(c) for c in chunks]
    n = len(arrs)
    ptrs = (ctypes.c_void_p * max(n, 1))(*[a.ctypes.data if a.size else None for a in arrs])
    lens = (ctypes.c_uint64 * max(n, 1))(*[a.size for a in arrs])
    sha = np.zeros(max(n, 1) * 32, dtype=np.uint8)
    hdr = np.zeros(max(n, 1) * 8, dtype=np.uint8) if headers else None
    N.check(lib.slime_rs_chunk_digests(ptrs, lens, n, sha.ctypes.data, hdr.ctypes.data if hdr is not None else None))
    return ([sha[32 * i:32 * i + 32].tobytes() for i in range(n)],
            [hdr[8 * i:8 * i + 8].tobytes() for i in range(n)] if hdr is not None else None)


def reconstruct(chunks: Sequence, indices: Sequence[int], mapping: int, size: int,
                out: np.ndarray | None = None, sha: bytes | None = None, device: int | None = None) -> np.ndarray:
    """The object's bytes (uint8 array) from `need` surviving chunks
    (reconstruct's slow path).  `out`: caller-owned uint8 buffer of >= size bytes.
    With `sha` (the file's SHA256) the result is verified and a mismatch
    raises BadHash, as reconstruct returns ErrBadHash (multi_store.go:244-249)."""
    arrs = [_bytes_view(c) for c in chunks]
    cb = arrs[0].size if arrs else 0
    if any(a.size != cb for a in arrs):
        raise ValueError("reconstruct: chunks must have equal length")
    ptrs = (ctypes.c_void_p * max(len(arrs), 1))(*[a.ctypes.data for a in arrs])
    idx = (ctypes.c_int * max(len(indices), 1))(*[int(i) for i in indices])
    if len(indices) != len(arrs):
        raise ValueError("reconstruct: one index per chunk")
    if out is None:
        out = np.empty(size, dtype=np.uint8)
    elif out.dtype != np.uint8 or not out.flags.c_contiguous or not out.flags.writeable or out.size < size:
        raise ValueError("reconstruct: out must be a writeable contiguous uint8 array of >= size bytes")
    out = out[:size]
    with N.on_device(device):
        if sha is not None:
            want = np.frombuffer(bytes(sha), dtype=np.uint8)
            if want.size != 32:
                raise ValueError("reconstruct: sha must be 32 bytes")
            N.check(lib.slime_rs_reconstruct_verify(ptrs, idx, len(arrs), cb, mapping & 0xFFFFFFFF, size,
                                                    out.ctypes.data if size else None, want.ctypes.data))
            return out
        N.check(lib.slime_rs_reconstruct(ptrs, idx, len(arrs), cb, mapping & 0xFFFFFFFF, size,
                                         out.ctypes.data if size else None))
    return out
