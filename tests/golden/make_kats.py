#!/usr/bin/env python3
"""Extract the reference's own known-answer tests into tests/golden/reference_kats.json.

Reads the Go test sources of encryptio/slime as TEXT (no Go toolchain is
needed or run) and records their literal inputs/expected outputs:

  internal/rs/matrix_test.go   TestVandermondeMatrix, TestParityMatrix
  internal/rs/vector_test.go   TestParityData (CreateParity KATs)
  internal/rs/gf/map_test.go   TestMapTrivial, TestMapTricky

The JSON it writes is data only (inputs and expected outputs). Re-run with
    python tests/golden/make_kats.py /root/reference
"""
from __future__ import annotations

import json
import os
import re
import sys


def _num(tok: str) -> int:
    tok = tok.strip()
    m = re.fullmatch(r"(\w+)\s*<<\s*(\w+)", tok)
    if m:
        return int(m.group(1), 0) << int(m.group(2), 0)
    return int(tok, 0)


def _list(body: str) -> list[int]:
    return [_num(t) for t in body.split(",") if t.strip()]


def _func_body(src: str, name: str) -> str:
    start = src.index(f"func {name}(")
    nxt = src.find("\nfunc ", start + 1)
    return src[start: nxt if nxt != -1 else len(src)]


def _matrix_cases(body: str, with_p=True):
    cases = []
    for m in re.finditer(r"D:\s*(\d+),\s*P:\s*(\d+),\s*M:\s*\[\]\[\]uint32\{(.*?)\n\t\t\t\},", body, re.S):
        rows = [_list(r) for r in re.findall(r"\[\]uint32\{([^}]*)\}", m.group(3))]
        cases.append({"d": int(m.group(1)), "p": int(m.group(2)), "m": rows})
    return cases


def main(ref_root: str) -> None:
    rs = os.path.join(ref_root, "internal", "rs")
    mt = open(os.path.join(rs, "matrix_test.go")).read()
    vt = open(os.path.join(rs, "vector_test.go")).read()
    gt = open(os.path.join(rs, "gf", "map_test.go")).read()

    out: dict = {"source": "encryptio/slime internal/rs test files (extracted as text by make_kats.py)"}
    out["vandermonde"] = _matrix_cases(_func_body(mt, "TestVandermondeMatrix"))
    out["parity_matrix"] = _matrix_cases(_func_body(mt, "TestParityMatrix"))

    pd = _func_body(vt, "TestParityData")
    cp = []
    for m in re.finditer(r"Data:\s*\[\]\[\]uint32\{(.*?)\n\t\t\t\},\s*Index:\s*(\d+),\s*Out:\s*\[\]uint32\{([^}]*)\}", pd, re.S):
        data = [_list(r) for r in re.findall(r"\[\]uint32\{([^}]*)\}", m.group(1))]
        cp.append({"data": data, "index": int(m.group(2)), "out": _list(m.group(3))})
    out["create_parity"] = cp

    mtb = _func_body(gt, "TestMapTrivial")
    trivial = []
    for m in re.finditer(r"\{\[\]byte\{([^}]*)\},\s*([^,]+),\s*\[\]uint32\{([^}]*)\}\}", mtb, re.S):
        trivial.append({"in": _list(m.group(1)), "n": _num(m.group(2)), "v": _list(m.group(3))})
    out["map_trivial"] = trivial

    mtk = _func_body(gt, "TestMapTricky")
    out["map_tricky"] = [_list(b) for b in re.findall(r"(?<!\])\[\]byte\{([^}]*)\}", mtk)]

    counts = {k: len(v) for k, v in out.items() if isinstance(v, list)}
    assert counts == {"vandermonde": 3, "parity_matrix": 3, "create_parity": 3, "map_trivial": 25,
                      "map_tricky": 6}, counts
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {dst}: {counts}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
