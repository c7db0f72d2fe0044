"""ORACLE — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT.

Second, independent CPU restatement of slime's internal/rs + internal/rs/gf
(reference /root/reference, encryptio/slime @ v0), written with Python
big integers (exact by construction) and a numpy column-vectorised
applyMatrix. It cross-checks the C restatement (oracle/rs_oracle.c) and
generates the golden vectors in tests/golden/. Only tests/, smoke() and
bench.py's cpu_baseline leg may import it; the product never does.

Parity pinning: checked against the reference's own known-answer tests
(tests/golden/reference_kats.json) in tests/test_oracle.py.
"""
from __future__ import annotations

import numpy as np

MaxVal = (1 << 32) - 5  # internal/rs/gf/map.go:7


class OraclePanic(Exception):
    """The reference panics; the oracle raises with the identical message."""


def minverse(x: int) -> int:
    """internal/rs/gf/gf.go:5-44: x^(p-2) mod p (the chain's exponent is exactly p-2)."""
    return pow(int(x), MaxVal - 2, MaxVal)


def raise_(x: int, n: int) -> int:
    """internal/rs/gf/gf.go:46-60 (recursive square-and-multiply; Raise(x,0)=1)."""
    if n == 0:
        return 1
    if x in (0, 1):
        return x
    v = raise_((x * x) % MaxVal, n // 2)
    if n % 2 == 1:
        v = (x * v) % MaxVal
    return v


def vandermonde(d: int, p: int) -> list[list[int]]:
    """internal/rs/matrix.go:8-22."""
    return [[raise_(j + 1, i) for j in range(d)] for i in range(d + p)]


def solve_sub_identity(m: list[list[int]]) -> None:
    """internal/rs/matrix.go:35-97: column Gauss-Jordan, same pivot rule and panics."""
    cols = len(m[0])
    for i in range(cols):
        if m[i][i] == 0:
            for j in range(i + 1, cols):
                if m[i][j] != 0:
                    for row in m:
                        row[i], row[j] = row[j], row[i]
                    break
            if m[i][i] == 0:
                raise OraclePanic("Couldn't ensure nonzero m[i][i]")
        if m[i][i] != 1:
            n = minverse(m[i][i])
            for row in m:
                row[i] = (row[i] * n) % MaxVal
            if m[i][i] != 1:
                raise OraclePanic("Couldn't ensure one m[i][i]")
        for j in range(cols):
            if j == i:
                continue
            if m[i][j] != 0:
                n = MaxVal - m[i][j]
                for row in m:
                    row[j] = (row[j] + (row[i] * n) % MaxVal) % MaxVal
                if m[i][j] != 0:
                    raise OraclePanic("Couldn't ensure zero m[i][j]")


def parity_matrix(d: int, p: int) -> list[list[int]]:
    """internal/rs/matrix.go:27-31."""
    m = vandermonde(d, p)
    solve_sub_identity(m)
    return m


def invert_matrix(m: list[list[int]]) -> list[list[int]]:
    """internal/rs/matrix.go:112-121."""
    d = len(m[0])
    c = [list(r) for r in m] + [[1 if j == i else 0 for j in range(d)] for i in range(d)]
    solve_sub_identity(c)
    return c[len(c) - d:]


def apply_matrix(mat, inp) -> list[np.ndarray]:
    """internal/rs/vector.go:90-102, vectorised over columns b with exact uint64 math.

    Each term is ((x*c) % p + o) % p in uint64, exactly as the reference.
    """
    ins = [np.asarray(v, dtype=np.uint64) for v in inp]
    outs = []
    P = np.uint64(MaxVal)
    for row in mat:
        o = np.zeros(len(ins[0]) if ins else 0, dtype=np.uint64)
        for j, x in enumerate(ins):
            o = ((x * np.uint64(row[j])) % P + o) % P
        outs.append(o.astype(np.uint32))
    return outs


def create_parity(data, index: int) -> np.ndarray:
    """internal/rs/vector.go:18-41."""
    for i in range(1, len(data)):
        if len(data[i]) != len(data[0]):
            raise OraclePanic("CreateParity called on data chunks of varying length")
    p = index - len(data) + 1 if index >= len(data) else 0
    mat = parity_matrix(len(data), p)
    return apply_matrix([mat[index]], data)[0]


def recover_data(chunks, indices) -> list[np.ndarray]:
    """internal/rs/vector.go:50-88."""
    if len(chunks) != len(indices):
        raise OraclePanic("RecoverData: len(chunks) != len(indices)")
    if len(chunks) == 0:
        raise OraclePanic("RecoverData: len(chunks) == 0")
    max_index = max(indices) if indices else -1
    if max_index == -1:
        raise OraclePanic("RecoverData: No indices given")
    mat = parity_matrix(len(chunks), max_index)
    have = [list(mat[i]) for i in indices]
    inv = invert_matrix(have)
    return apply_matrix(inv, chunks)


def _pack_be(data: bytes) -> np.ndarray:
    n = (len(data) + 3) // 4
    buf = bytes(data) + b"\x00" * (n * 4 - len(data))
    return np.frombuffer(buf, dtype=">u4").astype(np.uint32)


def map_to_gf_with(data: bytes, n: int) -> np.ndarray:
    """internal/rs/gf/map.go:74-98."""
    return _pack_be(data) ^ np.uint32(n)


def map_to_gf(data: bytes, candidates=()) -> tuple[int, np.ndarray]:
    """internal/rs/gf/map.go:15-67; the rand.Uint32() fallback draws from `candidates`."""
    out = _pack_be(data)
    if out.size == 0 or int(out.max()) < MaxVal:
        return 0, out
    cands = iter(candidates)
    n = 1 << 31
    while True:
        if int((out ^ np.uint32(n)).max()) < MaxVal:
            return n, out ^ np.uint32(n)
        try:
            n = int(next(cands))
        except StopIteration:
            raise OraclePanic("mapping fallback needed") from None


def map_from_gf(n: int, v) -> bytes:
    """internal/rs/gf/map.go:103-113."""
    return (np.asarray(v, dtype=np.uint32) ^ np.uint32(n)).astype(">u4").tobytes()


def split_vector(data: np.ndarray, count: int) -> list[np.ndarray]:
    """internal/store/multi/multi_store.go:271-299 (zero padded in the symbol domain)."""
    per = (len(data) + count - 1) // count
    flat = np.zeros(per * count, dtype=np.uint32)
    flat[: len(data)] = data
    return [flat[i * per:(i + 1) * per] for i in range(count)]
