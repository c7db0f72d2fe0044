#!/usr/bin/env python3
"""Per-launch duration of the C3 encode over a sustained run (after an idle
gap): does the kernel time drift with the chip's power/clock state?

    python tools/sustained.py [--seconds 8] [--idle 2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from slime_amd import device as D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--idle", type=float, default=2.0)
    args = ap.parse_args()
    need, total, L, nobj = 8, 12, 8 << 20, 128
    lay = D.layout_of(total, L)
    enc = D.Plan.encode(need, total)
    buf = torch.empty(nobj * total * L, dtype=torch.int32, device="cuda")
    D.fill_symbols(buf, 1)
    s = torch.cuda.current_stream()
    torch.cuda.synchronize()
    time.sleep(args.idle)
    n = int(args.seconds / 0.009)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    t0 = time.perf_counter()
    ev[0].record(s)
    for i in range(n):
        enc(buf, lay, buf, lay, L, nobj, dst_offset=need * L)
        ev[i + 1].record(s)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    d = [ev[i].elapsed_time(ev[i + 1]) for i in range(n)]
    win = max(1, n // 32)
    series = [round(sum(d[i:i + win]) / len(d[i:i + win]), 3) for i in range(0, n, win)]
    print(json.dumps({"launches": n, "wall_s": round(wall, 2), "first5": [round(x, 3) for x in d[:5]],
                      "window_means_ms": series, "min": round(min(d), 3), "max": round(max(d), 3)}))


if __name__ == "__main__":
    main()
