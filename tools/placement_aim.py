#!/usr/bin/env python3
"""The allocator's re-placement threshold (SLIME_RS_PLACEMENT_MIN_GBS, read
per allocation) as an A/B inside one process: rounds of a 48 GiB C3 batch
from slime_rs_device_alloc under each threshold in turn -- the allocation's
wall time, the probes it
made, the placement it kept, and the C3 encode / in-place repair kernels on
the kept buffer (median of 5 each) -- then the buffer back to the driver.
A pad allocation that changes size between rounds shifts where the next
buffer lands.

    python tools/placement_aim.py [--rounds 4 --thresholds 6100,6250]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from slime_amd import device as D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--thresholds", default="6100,6250")
    args = ap.parse_args()
    need, total, L, nobj = 8, 12, 8 << 20, 128
    lay = D.layout_of(total, L)
    enc = D.Plan.encode(need, total)
    dec = D.Plan.reconstruct(need, total, list(range(4, 12)), [0, 1, 2, 3]).set_outputs([0, 1, 2, 3])
    s = torch.cuda.current_stream()
    alg = nobj * 4 * L * total
    rows = []
    for r in range(args.rounds):
        for arm in args.thresholds.split(","):
            os.environ["SLIME_RS_PLACEMENT_MIN_GBS"] = arm
            pad = D.device_empty((1 + r % 3) * (1 << 28), torch.int32)  # 1-3 GiB: shift the placement
            t0 = time.perf_counter()
            buf = D.device_empty(nobj * total * L, torch.int32)
            alloc_s = time.perf_counter() - t0
            info = D.placement(buf)
            D.fill_symbols(buf, r)
            t = {"enc": [], "dec": []}
            for _ in range(6):
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                ev[0].record(s)
                enc(buf, lay, buf, lay, L, nobj, stream=s, dst_offset=need * L)
                ev[1].record(s)
                dec(buf, lay, buf, lay, L, nobj, stream=s)
                ev[2].record(s)
                torch.cuda.synchronize()
                t["enc"].append(ev[0].elapsed_time(ev[1]))
                t["dec"].append(ev[1].elapsed_time(ev[2]))
            e, d = statistics.median(t["enc"][1:]), statistics.median(t["dec"][1:])
            row = {"round": r, "threshold": arm, "alloc_s": round(alloc_s, 3), "kept": info["kept"],
                   "probes": [(p["placement"], round(p["probe_gbs"], 1)) for p in info["probes"]],
                   "enc_ms": round(e, 4), "dec_ms": round(d, 4),
                   "frac": round(alg / ((e + d) / 2 * 1e-3) / 8e12, 4)}
            print(json.dumps(row), flush=True)
            rows.append(row)
            del buf, pad
            torch.cuda.synchronize()
    for thr in sorted({r["threshold"] for r in rows}):
        fr = [r["frac"] for r in rows if r["threshold"] == thr]
        print(json.dumps({"threshold": thr, "rounds": len(fr), "frac_mean": round(statistics.mean(fr), 4),
                          "frac_min": min(fr), "frac_max": max(fr)}), flush=True)


if __name__ == "__main__":
    main()
