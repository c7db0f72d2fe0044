#!/usr/bin/env python3
"""Does the placement mode follow the batch's base offset inside its allocation?

One allocation of a C3 batch (128 objects x 12 shards x 8 Mi symbols, 48 GiB)
plus `--extra` MiB; the product encode is timed with the batch starting at
several byte offsets into it.  If the mode is a property of physical
address ranges, shifting the batch moves it.

    python tools/offset_probe.py [--offsets 0,2,4,...] [--extra 2048]
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
    ap.add_argument("--offsets", type=str, default="0,2,4,8,16,32,64,128,256,512,1024,1536")
    ap.add_argument("--extra", type=int, default=2048, help="MiB allocated past the batch")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    need, total, L, nobj = 8, 12, 8 << 20, 128
    n = nobj * total * L
    whole = torch.empty(n + (args.extra << 18), dtype=torch.int32, device="cuda")
    lay = D.layout_of(total, L)
    enc = D.Plan.encode(need, total)
    s = torch.cuda.current_stream()
    rows = []
    for off_mib in [int(x) for x in args.offsets.split(",")]:
        buf = whole[(off_mib << 18):(off_mib << 18) + n]
        D.fill_symbols(buf, 1)
        enc(buf, lay, buf, lay, L, nobj, dst_offset=need * L)
        ts = []
        for _ in range(args.reps):
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            enc(buf, lay, buf, lay, L, nobj, dst_offset=need * L)
            e.record(s)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(e))
        ms = statistics.median(ts)
        rows.append({"offset_mib": off_mib, "ms": round(ms, 3), "GBps": round(n * 4 / (ms * 1e-3) / 1e9, 1)})
        print(json.dumps(rows[-1]), flush=True)
    print(json.dumps({"base": hex(whole.data_ptr()), "rows": rows}))


if __name__ == "__main__":
    main()
