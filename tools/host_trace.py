#!/usr/bin/env python3
"""Per-call split of the object entry points' host pipeline (SLIME_RS_PIPE_TRACE):
write_chunks and reconstruct of one object, `--reps` times each, with the
library's trace lines (copy_in / enqueue split into h2d, launch, d2h / wait /
copy_out) on stderr and the median wall time per call on stdout.

    python tools/host_trace.py [--mib 64 --need 8 --total 12 --reps 8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ["SLIME_RS_PIPE_TRACE"] = "1"  # read once, when the library first runs a pipeline
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime per process: torch first)

from slime_amd import objects  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--need", type=int, default=8)
    ap.add_argument("--total", type=int, default=12)
    ap.add_argument("--reps", type=int, default=8)
    args = ap.parse_args()
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, size=args.mib << 20, dtype=np.uint8)
    cb = objects.chunk_size(data.size, args.need)
    chunks = [np.zeros(cb, dtype=np.uint8) for _ in range(args.total)]
    out = np.zeros(data.size, dtype=np.uint8)
    have = list(range(args.total - args.need, args.total))
    res = {}
    for what in ("write_chunks", "reconstruct"):
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            if what == "write_chunks":
                m, _ = objects.write_chunks(data, args.need, args.total, out=chunks, device=0)
            else:
                objects.reconstruct([chunks[i] for i in have], have, m, data.size, out=out, device=0)
            ts.append(time.perf_counter() - t0)
            print(f"--- {what} {ts[-1] * 1e3:.3f} ms", file=sys.stderr, flush=True)
        med = sorted(ts)[len(ts) // 2]
        res[what] = {"median_ms": round(med * 1e3, 3), "gibs": round(data.size / med / (1 << 30), 2)}
    res["verified"] = bool(np.array_equal(out, data))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
