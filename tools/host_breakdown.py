#!/usr/bin/env python3
"""Where the unchanged caller's time goes (host memory in and out, PCIe-inclusive).

multi_store.go calls the Go API call by call: MapToGF on the object (:526),
splitVector, r CreateParity calls (:528-531), one MapFromGF per chunk (:554) on
write; MapToGFWith per survivor (:224), RecoverData (:237), MapFromGF per data
row (:239) on read.  This times each call type at one object size through the
Python mirror of the Go API (slime_amd.rs / .gf), median of `--reps`.

    python tools/host_breakdown.py [--mib 64 --need 8 --total 12 --reps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime per process: torch first)

from slime_amd import gf, objects, rs  # noqa: E402


def med(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--need", type=int, default=8)
    ap.add_argument("--total", type=int, default=12)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    need, total, r = a.need, a.total, a.total - a.need
    rng = np.random.default_rng(0x5113E)
    data = rng.integers(0, 256, size=a.mib << 20, dtype=np.uint8)
    m, words = gf.MapToGF(data)
    parts = objects.split_vector(words, need)
    L = parts[0].size
    par = [np.zeros(L, dtype=np.uint32) for _ in range(r)]
    chunk = gf.MapFromGF(m, parts[0])
    have = list(range(r, total))
    code = parts + rs.CreateParities(parts, total)
    sym = [code[i] for i in have]
    rec = [np.zeros(L, dtype=np.uint32) for _ in range(need)]
    import ctypes
    from slime_amd import _native as N
    reused = np.zeros(words.size, dtype=np.uint32)
    mv = ctypes.c_uint32()

    def map_reused():
        N.check(N.lib.slime_gf_map_to_gf(data.ctypes.data, data.size, ctypes.byref(mv), reused.ctypes.data))

    t = {
        "MapToGF(object)": med(lambda: gf.MapToGF(data), a.reps),
        "MapToGF(object, reused output)": med(map_reused, a.reps),
        "CreateParity(1 row)": med(lambda: rs.CreateParity(parts, need, par[0]), a.reps),
        "MapFromGF(1 chunk)": med(lambda: gf.MapFromGF(m, parts[0]), a.reps),
        "MapToGFWith(1 chunk)": med(lambda: gf.MapToGFWith(chunk, m), a.reps),
        "RecoverData(need rows)": med(lambda: rs.RecoverData(sym, have, rec), a.reps),
        "CreateParities(r rows, batched)": med(lambda: rs.CreateParities(parts, total, par), a.reps),
    }
    write = t["MapToGF(object)"] + r * t["CreateParity(1 row)"] + total * t["MapFromGF(1 chunk)"]
    read = need * t["MapToGFWith(1 chunk)"] + t["RecoverData(need rows)"] + need * t["MapFromGF(1 chunk)"]
    gib = (a.mib << 20) / (1 << 30)
    print(json.dumps({"object_mib": a.mib, "need": need, "total": total,
                      "ms": {k: round(v * 1e3, 3) for k, v in t.items()},
                      "unchanged_write_ms": round(write * 1e3, 2), "unchanged_write_gibs": round(gib / write, 2),
                      "unchanged_read_ms": round(read * 1e3, 2), "unchanged_read_gibs": round(gib / read, 2)},
                     indent=1))


if __name__ == "__main__":
    main()
