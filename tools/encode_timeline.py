#!/usr/bin/env python3
"""Timeline of one fused byte encode call (slime_rs_encode_objects_phased):
which kernels and memsets a call enqueues and the gaps between them.

    rocprofv3 --kernel-trace -d gpurun_out/etl -o etl --output-format csv -- \\
        python3 tools/encode_timeline.py run [--need 10 --total 14 --mib 1024 --nobj 16]
    python3 tools/encode_timeline.py show gpurun_out/etl

`run` fills a batch as bench.py's byte leg does (256 B chunk strides), encodes
it `--reps` times back to back with HIP events around each call and prints the
event times; `show` lists, for the last call in the trace, every dispatch in
order with its duration and the idle gap before it, and sums kernels vs gaps.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(args):
    import torch

    from slime_amd import device as D
    need, total, nobj = args.need, args.total, args.nobj
    S = args.mib << 20
    L, cs, slot = D.slot_geometry(S, need, total, chunk_align=256)
    slots = D.device_empty(nobj * slot, torch.uint8, 0)
    D.fill_symbols(slots.view(torch.int32), 0xB17E5)
    enc = D.Plan.encode(need, total)
    mapping = torch.empty(nobj, dtype=torch.int32, device="cuda")
    status = torch.empty(nobj, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    D.encode_objects(enc, slots, slot, S, nobj, mapping, status, s, cs)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.reps + 1)]
    ev[0].record(s)
    for i in range(args.reps):
        D.encode_objects(enc, slots, slot, S, nobj, mapping, status, s, cs)
        ev[i + 1].record(s)
    torch.cuda.synchronize()
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(args.reps)]
    m = mapping.cpu().tolist()
    print(json.dumps({"shape": f"{need}/{total} {args.mib} MiB x {nobj}", "call_ms": [round(x, 4) for x in ms],
                      "switched": sum(1 for x in m if x != 0)}))


def show(d):
    path = glob.glob(os.path.join(d, "*kernel_trace.csv"))[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # calls begin with the status memset before the first encode pass: split at each first-pass kernel
    starts = [i for i, r in enumerate(rows) if "encode_bytes" in r["Kernel_Name"] and "redo" not in r["Kernel_Name"]]
    if len(starts) < 2:
        print("fewer than two calls in the trace")
        return
    a, b = starts[-2], starts[-1]
    # the memsets ahead of the first pass belong to the call
    while a > 0 and "encode_bytes" not in rows[a - 1]["Kernel_Name"] and "redo" not in rows[a - 1]["Kernel_Name"] \
            and "select" not in rows[a - 1]["Kernel_Name"]:
        a -= 1
    b0 = b
    while b0 > a and "encode_bytes" not in rows[b0 - 1]["Kernel_Name"] and "redo" not in rows[b0 - 1]["Kernel_Name"] \
            and "select" not in rows[b0 - 1]["Kernel_Name"]:
        b0 -= 1
    call = rows[a:b0]
    t0 = int(call[0]["Start_Timestamp"])
    prev_end = None
    busy = gaps = 0
    for r in call:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        busy += (e - s) / 1e3
        gaps += gap
        print(f"{(s - t0) / 1e3:10.1f} us  gap {gap:7.1f}  dur {(e - s) / 1e3:9.1f}  {r['Kernel_Name'][:90]}")
        prev_end = e
    print(json.dumps({"dispatches": len(call), "kernel_us": round(busy, 1), "gap_us": round(gaps, 1),
                      "span_us": round((prev_end - t0) / 1e3, 1)}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["run", "show"])
    ap.add_argument("dir", nargs="?")
    ap.add_argument("--need", type=int, default=10)
    ap.add_argument("--total", type=int, default=14)
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--nobj", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    if args.mode == "run":
        run(args)
    else:
        show(args.dir)


if __name__ == "__main__":
    main()
