#!/usr/bin/env python3
"""In-process A/B of the mid-object switch's second pass: re-encode of the
switched units (slime_rs_switch_bits(0)) against the top-bit parity
correction (1), alternated on the same buffers (one placement), with the
chunks of both compared.  Median encode ms (both passes) per mode.

    python tools/topbits_ab.py [--preset c5|c3 --rounds 8]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from slime_amd import _native as N  # noqa: E402
from slime_amd import device as D  # noqa: E402

SHAPES = {"c5": (10, 14, 1024, 16), "c3": (8, 12, 256, 128)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="c5")
    ap.add_argument("--rounds", type=int, default=8)
    args = ap.parse_args()
    need, total, mib, nobj = SHAPES[args.preset]
    S = mib << 20
    L, cs, slot = D.slot_geometry(S, need, total, chunk_align=256)
    slots = D.device_empty(nobj * slot, torch.uint8)
    words = slots.view(torch.int32)
    D.fill_symbols(words, 0xB17E5)
    enc = D.Plan.encode(need, total)
    mapping = torch.empty(nobj, dtype=torch.int32, device="cuda")
    status = torch.empty(nobj, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    for attempt in range(64):  # re-draw objects that need MapToGF's random fallback
        D.encode_objects(enc, slots, slot, S, nobj, mapping, status, s, cs)
        bad = status.nonzero().flatten().tolist()
        if not bad:
            break
        for o in bad:
            D.fill_symbols(words[o * slot // 4:(o * slot + need * cs) // 4], 0xB17E5 + (attempt + 1) * 2**32 + o)
    chunks = slots.view(nobj, total, cs)[:, :, : 4 * L]
    before = N.lib.slime_rs_switch_bits(-1)
    ref = None
    times = {0: [], 1: []}
    for r in range(args.rounds + 1):
        for mode in (0, 1):
            assert N.lib.slime_rs_switch_bits(mode) == 0
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            D.encode_objects(enc, slots, slot, S, nobj, mapping, status, s, cs)
            b.record(s)
            torch.cuda.synchronize()
            if ref is None:
                ref = chunks.clone()
            else:
                assert torch.equal(chunks, ref), (r, mode)
            if r:
                times[mode].append(a.elapsed_time(b))
    N.lib.slime_rs_switch_bits(before)
    ms = mapping.cpu().numpy().view("uint32")
    alg = nobj * 4 * L * total
    res = {"preset": args.preset, "mappings_1<<31": int((ms == 0x80000000).sum()), "nobj": nobj}
    for mode, name in ((0, "re-encode"), (1, "top-bit correction")):
        med = statistics.median(times[mode])
        res[name] = {"ms": round(med, 4), "frac": round(alg / med / 1e6 / 8000, 4), "min_ms": round(min(times[mode]), 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
