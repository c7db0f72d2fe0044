#!/usr/bin/env python3
"""Which traffic does the slow placement mode slow down?  ("Placement modes")

Allocates several C3-sized buffers (128 objects x 12 shards x 8 Mi symbols,
48 GiB each; each is its own hipMalloc segment, so each gets its own physical
placement) and times, on every buffer, the product encode and the same stripe
walk with XOR in place of the field math for these traffic mixes:
read 12 / read 8 / read 4 / write 4 / write 12 / read 8 + write 4.

    make placeprobe && python tools/placement_probe.py [--buffers 5] [--reps 3]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (owns the HIP runtime; load before our .so)

from slime_amd import device as D  # noqa: E402

MIXES = {0: ("read12", 12), 1: ("read8", 8), 4: ("read4", 4), 2: ("write4", 4), 5: ("write12", 12),
         3: ("read8+write4", 12)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--buffers", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--gx", type=int, default=4)
    ap.add_argument("--gy", type=int, default=128)
    args = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libplaceprobe.so"))
    lib.pp_launch.restype = ctypes.c_int
    lib.pp_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                              ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    need, total, L, nobj = 8, 12, 8 << 20, 128
    lay = D.layout_of(total, L)
    enc = D.Plan.encode(need, total)
    sink = torch.empty(args.gx * args.gy * 256, dtype=torch.int32, device="cuda")
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

    def timed(fn):
        fn()
        ts = []
        for _ in range(args.reps):
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            fn()
            e.record(s)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(e))
        return statistics.median(ts)

    rows = []
    for b, t in enumerate(bufs):
        row = {"buffer": b, "va": hex(t.data_ptr())}
        ms = timed(lambda: enc(t, lay, t, lay, L, nobj, dst_offset=need * L))
        row["encode"] = {"ms": round(ms, 3), "GBps": round(nobj * L * 4 * total / (ms * 1e-3) / 1e9, 1)}
        for mix, (name, nstripes) in MIXES.items():
            def go(mix=mix):
                rc = lib.pp_launch(mix, t.data_ptr(), total * L, L, L, nobj, args.gx, args.gy, sink.data_ptr(),
                                   ctypes.c_void_p(s.cuda_stream))
                assert rc == 0, rc
            ms = timed(go)
            row[name] = {"ms": round(ms, 3), "GBps": round(nobj * L * 4 * nstripes / (ms * 1e-3) / 1e9, 1)}
        rows.append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps({"buffers": len(bufs), "grid": [args.gx, args.gy], "per_buffer": rows}))


if __name__ == "__main__":
    main()
