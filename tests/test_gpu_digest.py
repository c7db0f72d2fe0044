"""write_chunks_digest / reconstruct verify on the GPU vs the oracle.

Chunks must equal the reference's writeChunks framing (multi_store.go:526-554,
via the C oracle) and every digest must equal SHA-256 (hashlib) and the
storedir chunk-file FNV-1a header (directory.go:548-553, oracle_fnv1a64) of
those chunks.  Kinds cover the three mapping outcomes of MapToGF (map.go:35-66):
0, 1<<31 (parity chunks rewritten after the speculative pass: the parity
hashers start over) and a random fallback mapping.
"""
from __future__ import annotations

import hashlib
import threading

import numpy as np
import pytest

from oracle import oracle_c as OC
from oracle import oracle_py as OP

pytestmark = pytest.mark.gpu


def _obj_bytes(rng, S, kind):
    b = bytearray(rng.integers(0, 256, size=S, dtype=np.uint8).tobytes())
    if kind == "high" and S >= 4:
        b[0:4] = b"\xff\xff\xff\xff"  # mapping 1<<31 (map.go:47)
    if kind == "fallback" and S >= 8:
        b[0:8] = b"\xff\xff\xff\xff\x7f\xff\xff\xff"  # neither 0 nor 1<<31
    return bytes(b)


def _oracle_chunks(obj: bytes, need: int, total: int, cands=()):
    rc, m, words = OC.map_to_gf(obj, list(cands))
    assert rc == 0
    parts = OP.split_vector(words, need)
    parity = [OC.create_parity(parts, need + i)[1] for i in range(total - need)]
    return m, [OC.map_from_gf(m, p) for p in parts + parity]


@pytest.mark.parametrize("need,total", [(2, 3), (4, 6), (8, 12), (10, 14), (17, 20), (8, 8)])
@pytest.mark.parametrize("S", [1, 5, 33, 4096, 100003, 3 * (8 << 20) + 13])
@pytest.mark.parametrize("kind", ["plain", "high", "fallback"])
def test_write_chunks_digest_vs_oracle(need, total, S, kind):
    from slime_amd import objects
    rng = np.random.default_rng(S * 7 + need)
    obj = _obj_bytes(rng, S, kind)
    m, chunks, shas, hdrs = objects.write_chunks_digest(obj, need, total, headers=True)
    if kind == "high" and S >= 4:
        assert m == 1 << 31
    m_ref, want = _oracle_chunks(obj, need, total, [m] if kind == "fallback" and S >= 8 else [])
    assert m == m_ref
    assert [c.tobytes() for c in chunks] == want
    for c, s, h in zip(want, shas, hdrs):
        assert (s, h) == OC.chunk_digests(c)


def test_write_chunks_digest_empty_object():
    from slime_amd import objects
    m, chunks, shas, hdrs = objects.write_chunks_digest(b"", 4, 6, headers=True)
    assert m == 0 and all(c.size == 0 for c in chunks)
    assert shas == [hashlib.sha256(b"").digest()] * 6
    assert hdrs == [OC.chunk_digests(b"")[1]] * 6


def test_write_chunks_digest_north_star_object():
    """8/12 with 64 MiB shards' object size class: a 64 MiB object (8 MiB chunks)."""
    from slime_amd import objects
    obj = np.random.default_rng(64).integers(0, 256, 64 << 20, dtype=np.uint8)
    m, chunks = objects.write_chunks(obj, 8, 12)
    m2, chunks2, shas, _ = objects.write_chunks_digest(obj, 8, 12)
    assert m == m2
    assert all(np.array_equal(a, b) for a, b in zip(chunks, chunks2))
    assert shas == [hashlib.sha256(c.tobytes()).digest() for c in chunks]


def test_write_chunks_digest_concurrent_callers():
    from slime_amd import objects
    rng = np.random.default_rng(5)
    objs = [_obj_bytes(rng, (3 << 20) + 1000 * i, "high" if i % 3 == 0 else "plain") for i in range(6)]
    errors = []

    def work(i):
        try:
            for _ in range(3):
                m, chunks, shas, _ = objects.write_chunks_digest(objs[i], 8, 12)
                assert shas == [hashlib.sha256(c.tobytes()).digest() for c in chunks]
                assert objects.reconstruct(chunks[4:], list(range(4, 12)), m, len(objs[i])).tobytes() == objs[i]
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(objs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors


@pytest.mark.parametrize("kind", ["plain", "high"])
def test_reconstruct_verify(kind):
    from slime_amd import _native as N
    from slime_amd import objects
    rng = np.random.default_rng(9)
    obj = _obj_bytes(rng, 1000003, kind)
    sha = hashlib.sha256(obj).digest()
    m, chunks = objects.write_chunks(obj, 8, 12)
    have = [0, 3, 5, 6, 8, 9, 10, 11]
    got = objects.reconstruct([chunks[i] for i in have], have, m, len(obj), sha=sha)
    assert got.tobytes() == obj
    bad = bytes([sha[0] ^ 1]) + sha[1:]
    with pytest.raises(N.BadHash):
        objects.reconstruct([chunks[i] for i in have], have, m, len(obj), sha=bad)
    corrupt = [c.copy() for c in chunks]
    corrupt[9][100] ^= 0x40  # a survivor flipped in storage: the rebuilt object no longer matches
    with pytest.raises(N.BadHash):
        objects.reconstruct([corrupt[i] for i in have], have, m, len(obj), sha=sha)


@pytest.mark.parametrize("need,total", [(4, 6), (8, 12), (8, 8), (17, 20)])
@pytest.mark.parametrize("S", [5, 4096, 100003, (8 << 20) + 4])
@pytest.mark.parametrize("kind", ["plain", "high"])
def test_write_chunks_zero_copy_data_chunks(need, total, S, kind):
    """alias=True: whole data chunks are views of the object and are not
    copied; every chunk still equals the reference's framing."""
    from slime_amd import objects
    rng = np.random.default_rng(S + need)
    obj = np.frombuffer(_obj_bytes(rng, S, kind), dtype=np.uint8).copy()
    m, chunks = objects.write_chunks(obj, need, total, alias=True)
    cb = objects.chunk_size(S, need)
    for j in range(need):
        if (j + 1) * cb <= S:
            assert np.shares_memory(chunks[j], obj)
    m_ref, want = _oracle_chunks(obj.tobytes(), need, total)
    assert m == m_ref and [c.tobytes() for c in chunks] == want
    m2, chunks2, shas, _ = objects.write_chunks_digest(obj, need, total, alias=True)
    assert m2 == m and [c.tobytes() for c in chunks2] == want
    assert shas == [hashlib.sha256(c).digest() for c in want]
