#!/usr/bin/env python3
"""Device-resident batches of many short objects on the matrix cores (tools
only): encode (all parity) and rebuild 4 erased shards per object of nobj
objects of L symbols a shard, HIP events around each launch, median of
--rounds; one JSON line per shape.

    python tools/short_objects.py --shapes 80/100,40/56 --L 64,512,2048 --nobj 4096
    python tools/short_objects.py --bytes 65536,262144 --nobj 1024   # byte objects: encode_objects/decode_objects
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

from slime_amd import device as D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="80/100,40/56")
    ap.add_argument("--L", default="64,512,2048")
    ap.add_argument("--nobj", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--bytes", default="", help="object sizes S in bytes (the byte path) instead of --L")
    a = ap.parse_args()
    if a.bytes:
        return byte_objects(a)
    for shape in a.shapes.split(","):
        need, total = (int(x) for x in shape.split("/"))
        for L in (int(x) for x in a.L.split(",")):
            lay = D.layout_of(total, L)
            buf = torch.empty(a.nobj * total * L, dtype=torch.int32, device="cuda")
            D.fill_symbols(buf, seed=L + need)
            enc = D.Plan.encode(need, total)
            erase = [0, 1, need, total - 1][: min(4, total - need + 1)]
            have = [i for i in range(total) if i not in erase][:need]
            dec = D.Plan.reconstruct(need, total, have, erase).set_outputs(erase)
            s = torch.cuda.current_stream()
            times = {"encode": [], "decode": []}
            for r in range(a.rounds + 1):
                for name, fn in (("encode", lambda: enc(buf, lay, buf, lay, L, a.nobj, dst_offset=need * L)),
                                 ("decode", lambda: dec(buf, lay, buf, lay, L, a.nobj))):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    fn()
                    e1.record(s)
                    e1.synchronize()
                    if r:
                        times[name].append(e0.elapsed_time(e1))
            alg = {"encode": a.nobj * 4 * L * total, "decode": a.nobj * 4 * L * (need + len(erase))}
            out = {"need": need, "total": total, "L": L, "nobj": a.nobj}
            for name in times:
                ms = statistics.median(times[name])
                out[name] = {"ms": round(ms, 4), "frac": round(alg[name] / ms / 1e-3 / 8e12, 4)}
            print(json.dumps(out), flush=True)
            del buf


def _time(fn, rounds):
    s = torch.cuda.current_stream()
    ts = []
    for r in range(rounds + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        fn()
        e1.record(s)
        e1.synchronize()
        if r:
            ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


def byte_objects(a):
    """encode_objects / decode_objects over nobj objects of S bytes (random
    bytes: every object maps with 0); the rate is over the object bytes plus
    the chunks written (encode) or read and rebuilt (decode)."""
    for shape in a.shapes.split(","):
        need, total = (int(x) for x in shape.split("/"))
        for S in (int(x) for x in a.bytes.split(",")):
            L, chunk, slot = D.slot_geometry(S, need, total)
            slots = torch.randint(0, 256, (a.nobj * slot,), dtype=torch.uint8, device="cuda")
            enc = D.Plan.encode(need, total)
            mapping = torch.empty(a.nobj, dtype=torch.int32, device="cuda")
            status = torch.empty(a.nobj, dtype=torch.int32, device="cuda")
            erase = [0, 1, need, total - 1][: min(4, total - need + 1)]
            have = [i for i in range(total) if i not in erase][:need]
            dec = D.Plan.reconstruct(need, total, have, erase).set_outputs(erase)
            t_enc = _time(lambda: D.encode_objects(enc, slots, slot, S, a.nobj, mapping, status), a.rounds)
            t_dec = _time(lambda: D.decode_objects(dec, slots, slot, L, a.nobj, mapping), a.rounds)
            alg_enc = a.nobj * (S + 4 * L * (total - need))
            alg_dec = a.nobj * 4 * L * (need + len(erase))
            print(json.dumps({"need": need, "total": total, "S": S, "nobj": a.nobj, "chunk_words": L,
                              "encode": {"ms": round(t_enc, 4), "frac": round(alg_enc / t_enc / 1e-3 / 8e12, 4)},
                              "decode": {"ms": round(t_dec, 4), "frac": round(alg_dec / t_dec / 1e-3 / 8e12, 4)}}),
                  flush=True)
            del slots


if __name__ == "__main__":
    main()
