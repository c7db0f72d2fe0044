"""Pin the oracle (test infrastructure) to the reference's own known-answer tests.

Every KAT in the reference's rs/gf test files (extracted verbatim into
tests/golden/reference_kats.json by tests/golden/make_kats.py) is checked
against BOTH restatements: oracle/rs_oracle.c (C, the reference's own `%`
arithmetic) and oracle/oracle_py.py (Python big integers).  The reference's
property tests are restated with a seeded RNG.
"""
import itertools
import random

import numpy as np
import pytest

from oracle import oracle_c as OC
from oracle import oracle_py as OP

P = OP.MaxVal


# internal/rs/matrix_test.go:8-55
def test_vandermonde_kats(kats):
    for case in kats["vandermonde"]:
        assert OC.vandermonde(case["d"], case["p"]).tolist() == case["m"]
        assert OP.vandermonde(case["d"], case["p"]) == case["m"]


# internal/rs/matrix_test.go:57-115
def test_parity_matrix_kats(kats):
    for case in kats["parity_matrix"]:
        assert OC.parity_matrix(case["d"], case["p"]).tolist() == case["m"]
        assert OP.parity_matrix(case["d"], case["p"]) == case["m"]


# internal/rs/vector_test.go:24-63
def test_create_parity_kats(kats):
    for case in kats["create_parity"]:
        rc, out = OC.create_parity(case["data"], case["index"])
        assert rc == 0 and out.tolist() == case["out"]
        assert OP.create_parity(case["data"], case["index"]).tolist() == case["out"]


# internal/rs/gf/map_test.go:9-76
def test_map_trivial_kats(kats):
    for case in kats["map_trivial"]:
        data = bytes(case["in"])
        rc, n, v = OC.map_to_gf(data)
        assert rc == 0 and n == case["n"] and v.tolist() == case["v"]
        n2, v2 = OP.map_to_gf(data)
        assert n2 == case["n"] and v2.tolist() == case["v"]
        assert OC.map_from_gf(n, v)[: len(data)] == data
        assert OP.map_from_gf(n, v)[: len(data)] == data


# internal/rs/gf/map_test.go:78-105 (the last case needs the random fallback)
def test_map_tricky_kats(kats):
    rng = random.Random(7)
    for case in kats["map_tricky"]:
        data = bytes(case)
        cands = [rng.getrandbits(32) for _ in range(64)]
        rc, n, v = OC.map_to_gf(data, cands)
        assert rc == 0
        assert all(int(x) < P for x in v)
        assert OC.map_from_gf(n, v)[: len(data)] == data
        n2, v2 = OP.map_to_gf(data, cands)
        assert (n2, v2.tolist()) == (n, v.tolist())


def test_map_tricky_last_case_needs_fallback(kats):
    # [FF FF FF FF 7F FF FF FF]: neither 0 nor 1<<31 works (map.go:64-66 loop).
    rc, _, _ = OC.map_to_gf(bytes(kats["map_tricky"][-1]), [])
    assert rc == 12


# internal/rs/gf/gf_test.go:8-26
def test_minverse_raise_property():
    rng = random.Random(1)
    for _ in range(1000):
        v = 0
        while v >= P or v == 0:
            v = rng.getrandbits(32)
        inv = OC.minverse(v)
        assert (v * inv) % P == 1
        assert inv == OC.raise_(v, P - 2) == OP.minverse(v) == OP.raise_(v, P - 2)


# internal/rs/matrix_test.go:117-168: every d-row subset of ParityMatrix(d,p) is invertible.
def test_parity_matrix_nonsingular():
    for d in range(1, 7):
        for p in range(0, 7):
            m = OC.parity_matrix(d, p)
            for pick in itertools.combinations(range(d + p), d):
                rc, _ = OC.invert_matrix(m[list(pick)])
                assert rc == 0, (d, p, pick)


def test_singular_panics():
    m = OC.parity_matrix(3, 2)
    rc, _ = OC.invert_matrix(m[[0, 0, 1]])
    assert rc == 5  # "Couldn't ensure nonzero m[i][i]"
    with pytest.raises(OP.OraclePanic, match=r"Couldn't ensure nonzero m\[i\]\[i\]"):
        OP.invert_matrix([list(m[0]), list(m[0]), list(m[1])])


# internal/rs/vector_test.go:65-113: random encode / erase / recover round trips.
@pytest.mark.parametrize("seed", range(12))
def test_parity_recovery_roundtrip(seed):
    rng = random.Random(seed)
    for L in range(1, 10):
        nd = rng.randrange(20)
        if nd == 0:
            continue
        data = [[rng.getrandbits(32) % P for _ in range(L)] for _ in range(nd)]
        npar = rng.randrange(20)
        parity = [OC.create_parity(data, nd + j)[1].tolist() for j in range(npar)]
        have = sorted(rng.sample(range(nd + npar), nd))
        chunks = [(data + parity)[i] for i in have]
        rc, rec = OC.recover_data(chunks, have)
        assert rc == 0 and [r.tolist() for r in rec] == data
        if nd <= 8:
            assert [r.tolist() for r in OP.recover_data(chunks, have)] == data


def test_c_and_python_apply_agree_on_edge_values():
    rng = np.random.default_rng(3)
    edges = np.array([0, 1, P - 1, P, P + 4, 0xFFFFFFFF, 0x80000000], dtype=np.uint32)
    for k in (1, 2, 5, 8, 16, 17):
        mat = rng.integers(0, P, size=(3, k), dtype=np.uint64).astype(np.uint32)
        mat[0, :] = P - 1
        ins = [rng.integers(0, 2**32, size=257, dtype=np.uint64).astype(np.uint32) for _ in range(k)]
        for x in ins:
            x[: edges.size] = edges
        a = OC.apply_matrix(mat, ins)
        b = OP.apply_matrix(mat.tolist(), ins)
        for u, v in zip(a, b):
            assert np.array_equal(u, v)


def test_golden_vectors_match_oracle(golden):
    for case in golden["parity_matrices"]:
        assert OC.parity_matrix(case["need"], case["total"] - case["need"]).tolist() == case["m"]
    for case in golden["encode"]:
        for i, row in enumerate(case["parity"]):
            assert OC.create_parity(case["data"], case["need"] + i)[1].tolist() == row
    for case in golden["decode"]:
        rc, rec = OC.recover_data(case["chunks"], case["have"])
        assert rc == 0 and [r.tolist() for r in rec] == case["data"]


def test_split_vector_padding():
    data = np.arange(1, 6, dtype=np.uint32)
    parts = OP.split_vector(data, 4)  # multi_store.go:271-299: perVector 2, zero-padded tail
    assert [p.tolist() for p in parts] == [[1, 2], [3, 4], [5, 0], [0, 0]]


def test_object_reps_matches_the_per_call_path():
    """oracle_object_reps (the CPU baseline's small-object timing loop, with the
    reference's matrix cache) computes what create_parity + recover_data do."""
    rng = np.random.default_rng(77)
    need, total, L = 8, 12, 129
    shards = np.zeros((total, L), dtype=np.uint32)
    shards[:need] = rng.integers(0, 2**32, size=(need, L), dtype=np.uint64).astype(np.uint32)
    want = shards.copy()
    OC.encode_object(want, need, total)
    have = [1, 4, 5, 6, 8, 9, 10, 11]
    rec = OC.object_reps(shards, need, total, have, 3)
    assert np.array_equal(shards[need:], want[need:])
    rc, ref = OC.recover_data([want[i] for i in have], have)
    assert rc == 0
    for a, b in zip(rec, ref):
        assert np.array_equal(a, b)
