"""ORACLE — TEST INFRASTRUCTURE ONLY. ctypes wrapper over oracle/liboracle.so.

The C restatement of internal/rs (oracle/rs_oracle.c), used as the checker by
tests/, __graft_entry__.smoke() and as bench.py's cpu_baseline ("port").
Never imported by the product (slime_amd/).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


def _load():
    if not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-C", HERE], check=True, capture_output=True)
    lib = ctypes.CDLL(LIB_PATH)
    V = ctypes.c_void_p
    sig = {
        "oracle_gf_minverse": (ctypes.c_uint32, [ctypes.c_uint32]),
        "oracle_gf_raise": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32]),
        "oracle_vandermonde": (None, [ctypes.c_int, ctypes.c_int, V]),
        "oracle_solve_sub_identity": (ctypes.c_int, [V, ctypes.c_int, ctypes.c_int]),
        "oracle_parity_matrix": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, V]),
        "oracle_invert_matrix": (ctypes.c_int, [V, ctypes.c_int, V]),
        "oracle_apply_matrix": (None, [V, ctypes.c_int, ctypes.c_int, V, V, ctypes.c_uint64]),
        "oracle_create_parity": (ctypes.c_int, [V, V, ctypes.c_int, ctypes.c_int, V]),
        "oracle_recover_data": (ctypes.c_int, [V, V, V, ctypes.c_int, ctypes.c_int, V]),
        "oracle_map_to_gf_with": (None, [V, ctypes.c_uint64, ctypes.c_uint32, V]),
        "oracle_map_to_gf": (ctypes.c_int, [V, ctypes.c_uint64, V, ctypes.c_int, V, V]),
        "oracle_map_from_gf": (None, [ctypes.c_uint32, V, ctypes.c_uint64, V]),
        "oracle_split_vector": (ctypes.c_uint64, [V, ctypes.c_uint64, ctypes.c_int, V]),
        "oracle_encode_object": (ctypes.c_int, [V, ctypes.c_int, ctypes.c_int, ctypes.c_uint64]),
        "oracle_object_reps": (ctypes.c_int, [V, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, V, V, ctypes.c_int]),
        "oracle_fnv1a64": (ctypes.c_uint64, [ctypes.c_uint64, V, ctypes.c_uint64]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    return lib


lib = _load()


def _ptrs(arrs):
    return (ctypes.c_void_p * max(len(arrs), 1))(*[a.ctypes.data for a in arrs])


def minverse(x: int) -> int:
    return int(lib.oracle_gf_minverse(x))


def raise_(x: int, n: int) -> int:
    return int(lib.oracle_gf_raise(x, n))


def vandermonde(d: int, p: int) -> np.ndarray:
    m = np.zeros((d + p, d), dtype=np.uint32)
    lib.oracle_vandermonde(d, p, m.ctypes.data)
    return m


def parity_matrix(d: int, p: int) -> np.ndarray:
    m = np.zeros((d + p, d), dtype=np.uint32)
    rc = lib.oracle_parity_matrix(d, p, m.ctypes.data)
    assert rc == 0, rc
    return m


def invert_matrix(m) -> tuple[int, np.ndarray]:
    a = np.ascontiguousarray(m, dtype=np.uint32)
    d = a.shape[0]
    inv = np.zeros((d, d), dtype=np.uint32)
    rc = lib.oracle_invert_matrix(a.ctypes.data, d, inv.ctypes.data)
    return rc, inv


def apply_matrix(mat, ins) -> list[np.ndarray]:
    m = np.ascontiguousarray(mat, dtype=np.uint32)
    ins = [np.ascontiguousarray(x, dtype=np.uint32) for x in ins]
    L = ins[0].size if ins else 0
    outs = [np.zeros(L, dtype=np.uint32) for _ in range(m.shape[0])]
    lib.oracle_apply_matrix(m.ctypes.data, m.shape[0], m.shape[1], _ptrs(ins), _ptrs(outs), L)
    return outs


def create_parity(data, index: int) -> tuple[int, np.ndarray]:
    arrs = [np.ascontiguousarray(x, dtype=np.uint32) for x in data]
    lens = (ctypes.c_uint64 * max(len(arrs), 1))(*[a.size for a in arrs])
    L = arrs[0].size if arrs else 0
    out = np.zeros(L, dtype=np.uint32)
    rc = lib.oracle_create_parity(_ptrs(arrs), lens, len(arrs), index, out.ctypes.data)
    return rc, out


def recover_data(chunks, indices) -> tuple[int, list[np.ndarray]]:
    arrs = [np.ascontiguousarray(x, dtype=np.uint32) for x in chunks]
    lens = (ctypes.c_uint64 * max(len(arrs), 1))(*[a.size for a in arrs])
    idx = (ctypes.c_int * max(len(indices), 1))(*indices)
    L = arrs[0].size if arrs else 0
    outs = [np.zeros(L, dtype=np.uint32) for _ in arrs]
    rc = lib.oracle_recover_data(_ptrs(arrs), lens, idx, len(arrs), len(indices), _ptrs(outs))
    return rc, outs


def map_to_gf(data: bytes, candidates=()) -> tuple[int, int, np.ndarray]:
    src = np.frombuffer(bytes(data), dtype=np.uint8)
    out = np.zeros((src.size + 3) // 4, dtype=np.uint32)
    cands = np.ascontiguousarray(list(candidates) or [0], dtype=np.uint32)
    m = ctypes.c_uint32(0)
    rc = lib.oracle_map_to_gf(src.ctypes.data, src.size, cands.ctypes.data, len(candidates), ctypes.byref(m),
                              out.ctypes.data)
    return rc, int(m.value), out


def map_to_gf_with(data: bytes, n: int) -> np.ndarray:
    src = np.frombuffer(bytes(data), dtype=np.uint8)
    out = np.zeros((src.size + 3) // 4, dtype=np.uint32)
    lib.oracle_map_to_gf_with(src.ctypes.data, src.size, n, out.ctypes.data)
    return out


def map_from_gf(n: int, v) -> bytes:
    w = np.ascontiguousarray(v, dtype=np.uint32)
    out = np.zeros(w.size * 4, dtype=np.uint8)
    lib.oracle_map_from_gf(n, w.ctypes.data, w.size, out.ctypes.data)
    return out.tobytes()


def encode_object(shards: np.ndarray, need: int, total: int) -> None:
    """In place on a C-contiguous [total][L] uint32 array: rows need..total-1 = parity."""
    assert shards.flags.c_contiguous and shards.dtype == np.uint32
    rc = lib.oracle_encode_object(shards.ctypes.data, need, total, shards.shape[1])
    assert rc == 0, rc


def object_reps(shards: np.ndarray, need: int, total: int, have, reps: int) -> list[np.ndarray]:
    """`reps` times the reference's per-object path with its matrix cache
    (r one-row CreateParity calls + one RecoverData), in C: the CPU baseline's
    per-call timing.  Returns the last RecoverData's rows."""
    assert shards.flags.c_contiguous and shards.dtype == np.uint32
    L = shards.shape[1]
    scratch = np.zeros((need, L), dtype=np.uint32)
    hv = (ctypes.c_int * need)(*have)
    rc = lib.oracle_object_reps(shards.ctypes.data, need, total, L, hv, scratch.ctypes.data, reps)
    assert rc == 0, rc
    return [scratch[t] for t in range(need)]


FNV64_OFFSET = 14695981039346656037


def fnv1a64(data, h: int = FNV64_OFFSET) -> int:
    """Go hash/fnv New64a over `data` continuing from h (oracle_fnv1a64)."""
    b = np.frombuffer(memoryview(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else \
        np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    return int(lib.oracle_fnv1a64(h, b.ctypes.data if b.size else None, b.size))


def chunk_digests(chunk) -> tuple[bytes, bytes]:
    """(SHA-256, chunk-file header) of one chunk as writeChunks and storedir
    produce them: store.DataV's sha256.Sum256 (internal/store/store.go:104-110;
    Python's hashlib, an independent SHA-256) and FNV-1a-64 over SHA-256 ‖ data,
    big-endian (storedir/directory.go:548-553)."""
    import hashlib
    raw = chunk.tobytes() if isinstance(chunk, np.ndarray) else bytes(chunk)
    sha = hashlib.sha256(raw).digest()
    return sha, fnv1a64(raw, fnv1a64(sha)).to_bytes(8, "big")
