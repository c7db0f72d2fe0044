#!/usr/bin/env python3
"""Which hardware counters separate the fast and slow placement modes of the
C3 encode?  Allocates several 48 GiB object buffers in one process (each is
its own hipMalloc segment, so each gets its own placement), times the encode
on each (HIP events), and prints the per-buffer times together with the
dispatch order, so a `rocprofv3 --pmc ... --kernel-trace` run of this script
can be split into fast-buffer and slow-buffer dispatches.

    python tools/placement_pmc.py [--buffers 5] [--reps 3]

Dispatch order: fill_kernel x buffers, then per buffer 1 + reps encodes.
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
    ap.add_argument("--buffers", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    need, total, L, nobj = 8, 12, 8 << 20, 128
    lay = D.layout_of(total, L)
    enc = D.Plan.encode(need, total)
    bufs = []
    for b in range(args.buffers):
        free, _ = torch.cuda.mem_get_info()
        if free < nobj * total * L * 4 + (8 << 30):
            break
        t = torch.empty(nobj * total * L, dtype=torch.int32, device="cuda")
        D.fill_symbols(t, b + 1)
        bufs.append(t)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    rows = []
    for b, t in enumerate(bufs):
        enc(t, lay, t, lay, L, nobj, dst_offset=need * L)  # warm
        times = []
        for _ in range(args.reps):
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            enc(t, lay, t, lay, L, nobj, dst_offset=need * L)
            e.record(s)
            torch.cuda.synchronize()
            times.append(a.elapsed_time(e))
        rows.append({"buffer": b, "va": hex(t.data_ptr()), "enc_ms": round(statistics.median(times), 3),
                     "all": [round(x, 3) for x in times]})
    print(json.dumps({"buffers": len(bufs), "reps": args.reps, "per_buffer": rows}))


if __name__ == "__main__":
    main()
