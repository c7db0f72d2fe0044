"""Python mirror of slime's ``internal/rs`` Go API over the MI355X C-ABI.

Same names, argument meaning and error behaviour as the reference
(/root/reference/internal/rs): where Go panics, these raise
``slime_amd.Panic`` carrying the reference's exact panic message.  Vectors are
1-D ``numpy.uint32`` arrays (Go ``[]uint32``); matrices are 2-D ``numpy.uint32``
arrays whose rows play the role of Go's ``[][]uint32`` rows.

Data-path calls (CreateParity, RecoverData, CreateParities) run on the GPU via
libslime_rs.so; matrix construction is exact host arithmetic.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np

from . import _native as N

lib = N.lib


def _vec(v) -> np.ndarray:
    return np.ascontiguousarray(v, dtype=np.uint32)


def _ptrs(arrays: Sequence[np.ndarray]):
    n = len(arrays)
    return (ctypes.c_void_p * max(n, 1))(*[a.ctypes.data for a in arrays])


def _lens(arrays: Sequence[np.ndarray]):
    n = len(arrays)
    return (ctypes.c_uint64 * max(n, 1))(*[a.size for a in arrays])


def _mat(rows: int, cols: int) -> np.ndarray:
    return np.zeros((rows, cols), dtype=np.uint32)


def vandermondeMatrix(d: int, p: int) -> np.ndarray:
    """internal/rs/matrix.go:8 — (d+p) x d, m[i][j] = (j+1)^i."""
    m = _mat(d + p, d)
    N.check(lib.slime_rs_vandermonde_matrix(d, p, m.ctypes.data))
    return m


def ParityMatrix(d: int, p: int) -> np.ndarray:
    """internal/rs/matrix.go:27 — systematic (d+p) x d code matrix."""
    m = _mat(d + p, d)
    N.check(lib.slime_rs_parity_matrix(d, p, m.ctypes.data))
    return m


def ParityMatrixCached(d: int, p: int) -> np.ndarray:
    """internal/rs/matrixcache.go:11 — shared, read-only (process-lifetime) matrix."""
    ptr = N.c_u32p()
    N.check(lib.slime_rs_parity_matrix_cached(d, p, ctypes.byref(ptr)))
    m = np.ctypeslib.as_array(ptr, shape=(d + p, d))
    m.flags.writeable = False
    return m


def solveSubIdentity(m: np.ndarray) -> None:
    """internal/rs/matrix.go:35 — in-place column Gauss-Jordan on a uint32 matrix."""
    if m.dtype != np.uint32 or not m.flags.c_contiguous:
        raise TypeError("solveSubIdentity needs a C-contiguous uint32 matrix")
    N.check(lib.slime_rs_solve_sub_identity(m.ctypes.data, m.shape[0], m.shape[1]))


def cloneMatrix(m) -> np.ndarray:
    """internal/rs/matrix.go:99 — a deep copy with one backing array."""
    return np.array(m, dtype=np.uint32, copy=True, order="C")


def invertMatrix(m) -> np.ndarray:
    """internal/rs/matrix.go:112 — inverse of a d x d matrix."""
    a = cloneMatrix(m)
    d = a.shape[1]
    inv = _mat(d, d)
    N.check(lib.slime_rs_invert_matrix(a.ctypes.data, d, inv.ctypes.data))
    return inv


def CreateParity(data: Sequence, index: int, out=None) -> np.ndarray:
    """internal/rs/vector.go:18 — code row `index` of `data`, computed on the GPU.

    Reuses `out` when it holds at least len(data[0]) elements (Go's cap rule)."""
    arrays = [_vec(d) for d in data]
    n = len(arrays)
    L = arrays[0].size if n else 0
    if n and all(a.size == L for a in arrays):
        if out is not None and isinstance(out, np.ndarray) and out.dtype == np.uint32 and out.size >= L \
                and out.flags.c_contiguous:
            res = out[:L]
        else:
            res = np.zeros(L, dtype=np.uint32)
        out_ptr = res.ctypes.data
    else:
        res, out_ptr = None, None
    N.check(lib.slime_rs_create_parity(_ptrs(arrays), _lens(arrays), n, index, out_ptr))
    return res


def _outs(outs, n: int, L: int) -> list[np.ndarray]:
    """Caller-supplied result rows (uint32, contiguous, >= L symbols) are
    written in place and returned as [:L] views; otherwise fresh rows."""
    if outs is None:
        return [np.zeros(L, dtype=np.uint32) for _ in range(n)]
    if len(outs) != n:
        raise ValueError(f"expected {n} output rows, got {len(outs)}")
    res = []
    for o in outs:
        if not (isinstance(o, np.ndarray) and o.dtype == np.uint32 and o.flags.c_contiguous
                and o.flags.writeable and o.size >= L):
            raise ValueError("output rows must be writeable contiguous uint32 arrays of at least L symbols")
        res.append(o[:L])
    return res


def CreateParities(data: Sequence, total: int, outs: Sequence[np.ndarray] | None = None) -> list[np.ndarray]:
    """All total-len(data) parity rows in one GPU pass (batched multi_store.go:528-531)."""
    arrays = [_vec(d) for d in data]
    L = arrays[0].size if arrays else 0
    outs = _outs(outs, max(total - len(arrays), 0), L)
    N.check(lib.slime_rs_create_parities(_ptrs(arrays), _lens(arrays), len(arrays), total, _ptrs(outs)))
    return outs


def RecoverData(chunks: Sequence, indices: Sequence[int],
                outs: Sequence[np.ndarray] | None = None) -> list[np.ndarray]:
    """internal/rs/vector.go:50 — all len(chunks) data rows from any len(chunks) code rows."""
    arrays = [_vec(c) for c in chunks]
    idx = (ctypes.c_int * max(len(indices), 1))(*[int(i) for i in indices])
    L = arrays[0].size if arrays else 0
    outs = _outs(outs, len(arrays), L)
    N.check(lib.slime_rs_recover_data(_ptrs(arrays), _lens(arrays), len(arrays), idx, len(indices), _ptrs(outs)))
    return outs
