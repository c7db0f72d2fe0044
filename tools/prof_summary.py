#!/usr/bin/env python3
"""Per-kernel durations of the full-size launches in a rocprofv3 kernel trace
of `bench.py`.  The stats CSV averages every launch of a kernel name, and the
default bench command also runs the host leg (hundreds of small windowed
launches of the same apply kernel) and the placement / allocator probes; this
splits the C3-sized launches (over --min-ms) out so their average can be set
against the bench line's own kernel_ms.

    python tools/prof_summary.py <dir with bench_kernel_trace.csv> [--min-ms 5]
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min-ms", type=float, default=5.0)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(os.path.join(args.dir, "bench_kernel_trace.csv"))))
    by = {}
    for r in rows:
        ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        name = r["Kernel_Name"].split("(")[0]
        by.setdefault(name, []).append(ms)
    out = {}
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        big = [x for x in v if x >= args.min_ms]
        if not big:
            continue
        out[name] = {"launches": len(v), "full_size_launches": len(big), "mean_ms": round(statistics.mean(big), 4),
                     "median_ms": round(statistics.median(big), 4), "min_ms": round(min(big), 4),
                     "max_ms": round(max(big), 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
