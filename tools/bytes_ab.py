#!/usr/bin/env python3
"""In-process A/B of the work schedules of the fused byte kernels (the bench's
object_bytes_path): same buffers, schedules alternated round by round with
slime_rs_kernel_schedule, so allocation placement cannot bias the result.

    python tools/bytes_ab.py [--need 8 --total 12 --object-mib 256 --objects 128 --rounds 5]
"""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--need", type=int, default=8)
    ap.add_argument("--total", type=int, default=12)
    ap.add_argument("--object-mib", type=int, default=256)
    ap.add_argument("--objects", type=int, default=128)
    ap.add_argument("--erase", type=str, default="0,1,2,3")
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    need, total, nobj = args.need, args.total, args.objects
    erase = [int(x) for x in args.erase.split(",")]
    S = args.object_mib << 20
    L, chunk, slot = D.slot_geometry(S, need, total)
    slots = torch.empty(nobj * slot, dtype=torch.uint8, device="cuda")
    D.fill_symbols(slots.view(torch.int32), 0xB17E5)
    enc = D.Plan.encode(need, total)
    have = [i for i in range(total) if i not in erase][:need]
    dec = D.Plan.reconstruct(need, total, have, erase).set_outputs(erase)
    mapping = torch.empty(nobj, dtype=torch.int32, device="cuda")
    status = torch.empty(nobj, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    words = slots.view(torch.int32)
    redraws = 0
    for attempt in range(64):  # objects needing MapToGF's random fallback are re-drawn (as bench.py does)
        D.encode_objects(enc, slots, slot, S, nobj, mapping, status, s)
        bad = status.nonzero().flatten().tolist()
        if not bad:
            break
        for o in bad:
            D.fill_symbols(words[o * slot // 4:(o * slot + S) // 4], 0xB17E5 + (attempt + 1) * 2**32 + o)
        redraws += len(bad)
    truth = slots.view(nobj, slot)[:, : total * chunk].view(nobj, total, chunk)[:, erase, :].clone()
    before = N.lib.slime_rs_kernel_schedule(-1)
    times = {0: {"enc": [], "dec": []}, 1: {"enc": [], "dec": []}}
    ok = True
    for r in range(args.rounds + 1):
        for sched in (0, 1):
            assert N.lib.slime_rs_kernel_schedule(sched) == 0
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record(s)
            D.encode_objects(enc, slots, slot, S, nobj, mapping, status, s)
            ev[1].record(s)
            D.decode_objects(dec, slots, slot, L, nobj, mapping, s)
            ev[2].record(s)
            torch.cuda.synchronize()
            if r:  # round 0 warms both forms up
                times[sched]["enc"].append(ev[0].elapsed_time(ev[1]))
                times[sched]["dec"].append(ev[1].elapsed_time(ev[2]))
            got = slots.view(nobj, slot)[:, : total * chunk].view(nobj, total, chunk)[:, erase, :]
            ok = ok and bool(torch.equal(got, truth)) and int(status.sum().item()) == 0
    N.lib.slime_rs_kernel_schedule(before)
    ms = mapping.cpu().numpy().view("uint32")
    out = {"shape": f"{need}/{total} {args.object_mib} MiB x {nobj}", "verified": ok, "fallback_redraws": redraws,
           "objects_mapped_1<<31": int((ms == 0x80000000).sum())}
    for sched, name in ((0, "static"), (1, "dynamic")):
        e, d = statistics.median(times[sched]["enc"]), statistics.median(times[sched]["dec"])
        out[name] = {"encode_both_passes_ms": round(e, 4), "decode_ms": round(d, 4),
                     "object_gibs": round(2 * nobj * S / 2**30 / ((e + d) * 1e-3), 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
