#!/usr/bin/env python3
"""In-process A/B of the fused byte encode's second pass through the product
API (slime_rs_encode_objects_phased): slime_rs_switch_bits(2) re-encodes the
units a switched object encoded with mapping 0, (1) corrects them from the
top bits the first pass stored.  One allocation per shape, the bench's data
and fallback re-draws, modes alternating; the chunks of both modes must be
equal byte for byte.  Prints median ms of pass 0, the second pass and the
whole encode per mode.

    python tools/topbits_ab.py [--shapes c5,c3 --rounds 8]
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

SHAPES = {"c5": (10, 14, 1024, 16), "c3": (8, 12, 256, 128), "c5_512": (10, 14, 512, 32)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="c5,c3")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--seed", type=int, default=0xB17E5)
    args = ap.parse_args()
    before = N.lib.slime_rs_switch_bits(-1)
    out = {}
    stream = torch.cuda.current_stream()
    for shape in args.shapes.split(","):
        need, total, mib, nobj = SHAPES[shape]
        S = mib << 20
        L, cs, slot = D.slot_geometry(S, need, total, chunk_align=256)
        slots = D.device_empty(nobj * slot, torch.uint8)
        words = slots.view(torch.int32)
        D.fill_symbols(words, args.seed)
        enc = D.Plan.encode(need, total)
        mapping = torch.empty(nobj, dtype=torch.int32, device="cuda")
        status = torch.empty(nobj, dtype=torch.int32, device="cuda")
        for attempt in range(64):  # the bench's re-draw of objects MapToGF would map at random
            D.encode_objects(enc, slots, slot, S, nobj, mapping, status, stream, cs)
            bad = status.nonzero().flatten().tolist()
            if not bad:
                break
            for o in bad:
                D.fill_symbols(words[o * slot // 4:(o * slot + need * cs) // 4], args.seed + (attempt + 1) * 2**32 + o)
        times, ref = {}, None
        for r in range(args.rounds + 1):
            for mode, name in ((2, "re-encode"), (1, "top-bit correction")):
                assert N.lib.slime_rs_switch_bits(mode) == 0
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                ev[1].record(stream)
                ev[0].record(stream)
                D.encode_objects(enc, slots, slot, S, nobj, mapping, status, stream, cs, phase_event=ev[1])
                ev[2].record(stream)
                torch.cuda.synchronize()
                assert int(status.sum().item()) == 0
                par = slots.view(nobj, slot)[:, need * cs: total * cs]
                if ref is None:
                    ref = par.clone()
                else:
                    assert torch.equal(par, ref), (shape, name)
                if r:
                    t = times.setdefault(name, {"pass0": [], "second": [], "encode": []})
                    t["pass0"].append(ev[0].elapsed_time(ev[1]))
                    t["second"].append(ev[1].elapsed_time(ev[2]))
                    t["encode"].append(ev[0].elapsed_time(ev[2]))
        alg = nobj * 4 * L * total
        res = {"switched": int((mapping != 0).sum().item()), "nobj": nobj}
        for name, t in times.items():
            e = statistics.median(t["encode"])
            res[name] = {k: round(statistics.median(v), 4) for k, v in t.items()}
            res[name]["frac"] = round(alg / (e * 1e-3) / 8e12, 4)
            print(shape, name, res[name], flush=True)
        out[shape] = res
        del slots, words, ref
        torch.cuda.empty_cache()
    N.lib.slime_rs_switch_bits(before)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
