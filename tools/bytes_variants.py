#!/usr/bin/env python3
"""A/B the speculative byte-domain encode pass (tools/bytes_variants.hip) at C3,
in one process and on one allocation, next to the product symbol-domain
encode as the reference point.  Outputs are checked against the product's.

    make bytesvar && python tools/bytes_variants.py
"""
from __future__ import annotations

import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from slime_amd import device as D  # noqa: E402

NAMES = {0: "U4 fast flags (product)", 1: "U4 fast noflags", 2: "U4 nofast flags", 3: "U2 fast flags",
         4: "U1 fast flags", 5: "U2 fast noflags", 6: "U1 fast noflags"}


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libbytesvar.so"))
    lib.bv_encode.restype = ctypes.c_int
    lib.bv_encode.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                              ctypes.c_uint32, ctypes.c_uint32] + [ctypes.c_void_p] * 4 + \
        [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    need, total, nobj, S = 8, 12, 128, 256 << 20
    L, chunk, slot = D.slot_geometry(S, need, total)
    slots = torch.empty(nobj * slot, dtype=torch.uint8, device="cuda")
    words = slots.view(torch.int32)
    D.fill_symbols(words, 5)
    enc = D.Plan.encode(need, total)
    mapping = torch.zeros(nobj, dtype=torch.int32, device="cuda")
    status = torch.zeros(nobj, dtype=torch.int32, device="cuda")
    D.encode_objects(enc, slots, slot, S, nobj, mapping, status)
    torch.cuda.synchronize()
    ref = slots.view(nobj, slot)[:, need * chunk:].clone()
    coeff = np.zeros((total - need, 16), dtype=np.uint32)
    coeff[:, :need] = enc.coefficients()
    c_t = torch.from_numpy(coeff.view(np.int32).reshape(-1)).cuda()
    oi = torch.arange(total - need, dtype=torch.int32, device="cuda")
    flags = torch.zeros(nobj, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    lay = D.layout_of(total, L)

    def t(fn):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        fn()
        b.record(s)
        torch.cuda.synchronize()
        return a.elapsed_time(b)

    res = {}
    for _ in range(3):
        res.setdefault("sym encode", []).append(t(lambda: enc(words, lay, words, lay, L, nobj, dst_offset=need * L)))
        for v in NAMES:
            for blocks in (256, 512, 1024):
                gx = max(1, blocks // nobj)
                res.setdefault((v, blocks), []).append(t(lambda: lib.bv_encode(
                    v, ctypes.c_void_p(slots.data_ptr()), slot, L, S, nobj, total - need, ctypes.c_void_p(c_t.data_ptr()),
                    ctypes.c_void_p(oi.data_ptr()), ctypes.c_void_p(flags.data_ptr()),
                    ctypes.c_void_p(mapping.data_ptr()), gx, nobj, ctypes.c_void_p(s.cuda_stream))))
    # speculative pass writes the mapping-0 parity; objects remapped to 1<<31 differ from ref by design
    m0 = (mapping == 0).cpu()
    ok = bool(torch.equal(slots.view(nobj, slot)[:, need * chunk:][m0.cuda()], ref[m0.cuda()]))
    out = {"sym_encode_ms": round(statistics.median(res.pop("sym encode")), 3), "mapping0_outputs_match": ok}
    out["variants"] = sorted(({"variant": NAMES[v], "blocks": b, "ms": round(statistics.median(x), 3)}
                              for (v, b), x in res.items()), key=lambda r: r["ms"])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
