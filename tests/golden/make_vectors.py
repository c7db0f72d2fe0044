#!/usr/bin/env python3
"""Generate tests/golden/vectors.json — small golden vectors for the RS codec.

Produced by the Python big-int restatement (oracle/oracle_py.py) and
cross-checked against the C restatement (oracle/rs_oracle.c) before writing.
Both oracles are pinned to the reference's own KATs by tests/test_oracle.py.
Re-run:  python tests/golden/make_vectors.py
"""
from __future__ import annotations

import itertools
import json
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle_c as OC  # noqa: E402
from oracle import oracle_py as OP  # noqa: E402

P = OP.MaxVal
EDGE = [0, 1, 2, P - 2, P - 1, P, P + 1, P + 4, 0xFFFFFFFF, 0x7FFFFFFF, 0x80000000]


def vec(rng: random.Random, L: int, edges: bool) -> list[int]:
    v = [rng.getrandbits(32) % P for _ in range(L)]
    if edges:
        for i in range(min(L, len(EDGE))):
            v[rng.randrange(L)] = EDGE[i]
    return v


def main() -> None:
    rng = random.Random(0x5113E)
    out: dict = {"generator": "tests/golden/make_vectors.py (oracle_py, cross-checked with oracle_c)", "p": P}

    shapes = [(2, 3), (3, 5), (4, 6), (6, 8), (8, 12), (10, 14), (7, 17), (17, 20)]
    out["parity_matrices"] = []
    for need, total in shapes:
        m = OP.parity_matrix(need, total - need)
        assert np.array_equal(np.array(m, dtype=np.uint32), OC.parity_matrix(need, total - need))
        out["parity_matrices"].append({"need": need, "total": total, "m": m})

    out["inverses"] = []
    sets = [(4, 6, list(s)) for s in itertools.combinations(range(6), 4)]
    sets += [(8, 12, list(range(4, 12))), (8, 12, [1, 2, 4, 5, 6, 7, 9, 10]), (8, 12, [0, 1, 2, 3, 8, 9, 10, 11]),
             (10, 14, list(range(4, 14))), (2, 3, [1, 2]), (2, 3, [0, 2])]
    for need, total, have in sets:
        full = OP.parity_matrix(need, total - need)
        inv = OP.invert_matrix([full[i] for i in have])
        rc, inv_c = OC.invert_matrix([full[i] for i in have])
        assert rc == 0 and np.array_equal(np.array(inv, dtype=np.uint32), inv_c)
        out["inverses"].append({"need": need, "total": total, "have": have, "inv": inv})

    out["encode"] = []
    for need, total in [(2, 3), (4, 6), (8, 12), (10, 14), (3, 5), (17, 20)]:
        for L in (1, 3, 5, 17, 64):
            data = [vec(rng, L, edges=True) for _ in range(need)]
            parity = [OP.create_parity(data, need + i).tolist() for i in range(total - need)]
            for i in range(total - need):
                rc, pc = OC.create_parity(data, need + i)
                assert rc == 0 and pc.tolist() == parity[i]
            out["encode"].append({"need": need, "total": total, "L": L, "data": data, "parity": parity})

    out["decode"] = []
    for need, total, have in [(4, 6, [1, 2, 4, 5]), (4, 6, [0, 3, 4, 5]), (8, 12, list(range(4, 12))),
                              (8, 12, [1, 2, 4, 5, 6, 7, 9, 10]), (10, 14, [0, 2, 4, 6, 8, 9, 10, 11, 12, 13]),
                              (2, 3, [2, 1])]:
        L = 13
        data = [vec(rng, L, edges=False) for _ in range(need)]
        code = data + [OP.create_parity(data, need + i).tolist() for i in range(total - need)]
        chunks = [code[i] for i in have]
        rec = [r.tolist() for r in OP.recover_data(chunks, have)]
        assert rec == data
        rc, rec_c = OC.recover_data(chunks, have)
        assert rc == 0 and [r.tolist() for r in rec_c] == rec
        out["decode"].append({"need": need, "total": total, "have": have, "chunks": chunks, "data": rec})

    out["map"] = []
    samples = [b"", b"\x00", b"\xff", b"\x12\x34\x56", b"\xff\xff\xff\xfb", b"\x7f\xff\xff\xfb\x00",
               b"\xff\xff\xff\xff\x01\x02", bytes(range(256)), bytes(rng.getrandbits(8) for _ in range(37))]
    for s in samples:
        n, words = OP.map_to_gf(s)
        rc, nc, wc = OC.map_to_gf(s)
        assert rc == 0 and nc == n and wc.tolist() == words.tolist()
        out["map"].append({"bytes": list(s), "n": n, "words": words.tolist(),
                           "back": list(OP.map_from_gf(n, words))})

    dst = os.path.join(ROOT, "tests", "golden", "vectors.json")
    with open(dst, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(f"wrote {dst} ({os.path.getsize(dst)} bytes)")


if __name__ == "__main__":
    main()
