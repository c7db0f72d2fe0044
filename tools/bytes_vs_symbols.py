#!/usr/bin/env python3
"""Fused byte-domain kernels vs symbol-domain kernels on the SAME allocation
(C3 shape): separates kernel cost from the allocation's placement mode.

    python tools/bytes_vs_symbols.py
"""
from __future__ import annotations

import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from slime_amd import device as D  # noqa: E402


def timed(fn, n=5):
    s = torch.cuda.current_stream()
    t = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        fn()
        b.record(s)
        torch.cuda.synchronize()
        t.append(a.elapsed_time(b))
    return round(statistics.median(t), 3)


def main():
    need, total, nobj, S = 8, 12, 128, 256 << 20
    L, chunk, slot = D.slot_geometry(S, need, total)
    slots = torch.empty(nobj * slot, dtype=torch.uint8, device="cuda")
    words = slots.view(torch.int32)
    D.fill_symbols(words, 5)
    lay = D.layout_of(total, L)
    enc = D.Plan.encode(need, total)
    erase = [0, 1, 2, 3]
    have = list(range(4, 12))
    dec = D.Plan.reconstruct(need, total, have, erase).set_outputs(erase)
    mapping = torch.zeros(nobj, dtype=torch.int32, device="cuda")
    status = torch.zeros(nobj, dtype=torch.int32, device="cuda")
    D.encode_objects(enc, slots, slot, S, nobj, mapping, status)
    torch.cuda.synchronize()
    nmap = int((mapping != 0).sum().item())
    out = {
        "sym_encode_ms": timed(lambda: enc(words, lay, words, lay, L, nobj, dst_offset=need * L)),
        "bytes_encode_ms": timed(lambda: D.encode_objects(enc, slots, slot, S, nobj, mapping, status)),
        "sym_decode_ms": timed(lambda: dec(words, lay, words, lay, L, nobj)),
        "bytes_decode_ms": timed(lambda: D.decode_objects(dec, slots, slot, L, nobj, mapping)),
        "objects_remapped_1<<31": nmap,
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
