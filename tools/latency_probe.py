"""Latency floor of one small host call on this box (tools only).

Times, median of many calls, in microseconds:
- a pinned 4 KiB H2D copy + stream sync; the same D2H; an empty-ish kernel + sync;
- the chain H2D -> kernel -> D2H with one sync (what a one-window host call needs);
- the library's CreateParity / RecoverData / write_chunks / reconstruct at 4 KiB and 64 KiB,
  each with its pipeline split (slime_rs_host_stats).
Usage: python tools/latency_probe.py
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from slime_amd import _native as N  # noqa: E402
from slime_amd import gf, objects, rs  # noqa: E402


def med_us(fn, reps=200):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return round(ts[len(ts) // 2] * 1e6, 1)


def main():
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream()
    h = torch.empty(1024, dtype=torch.int32).pin_memory()
    d = torch.empty(1024, dtype=torch.int32, device=dev)
    out = {}
    with torch.cuda.stream(s):
        out["h2d_4k_sync"] = med_us(lambda: (d.copy_(h, non_blocking=True), s.synchronize()))
        out["d2h_4k_sync"] = med_us(lambda: (h.copy_(d, non_blocking=True), s.synchronize()))
        out["kernel_sync"] = med_us(lambda: (d.add_(1), s.synchronize()))
        out["h2d_kernel_d2h_sync"] = med_us(lambda: (d.copy_(h, non_blocking=True), d.add_(1),
                                                     h.copy_(d, non_blocking=True), s.synchronize()))
    need, total, erase = 8, 12, [0, 1, 2, 3]
    have = [i for i in range(total) if i not in erase][:need]
    rng = np.random.default_rng(1)
    for kib in (4, 64):
        data = rng.integers(0, 256, size=kib << 10, dtype=np.uint8)
        cb = objects.chunk_size(data.size, need)
        chunks = [np.zeros(cb, dtype=np.uint8) for _ in range(total)]
        o = np.zeros(data.size, dtype=np.uint8)
        box = {}
        row = {}

        def timed(name, fn):
            N.host_stats(reset=True)
            row[name] = med_us(fn, 100)
            st = N.host_stats(reset=True)
            c = max(1, st["calls"])
            row[name + "_split_us"] = {k: round(st[k] / c, 1) for k in ("copy_in_us", "enqueue_us", "wait_us",
                                                                        "copy_out_us", "total_us")}
        timed("write_chunks", lambda: box.update(m=objects.write_chunks(data, need, total, out=chunks)[0]))
        surv = [chunks[i] for i in have]
        timed("reconstruct", lambda: objects.reconstruct(surv, have, box["m"], data.size, out=o))
        m, words = gf.MapToGF(data)
        parts = objects.split_vector(words, need)
        par = np.zeros(parts[0].size, dtype=np.uint32)
        timed("create_parity", lambda: rs.CreateParity(parts, need, par))
        sym = [gf.MapToGFWith(chunks[i], m) for i in have]
        rec = [np.zeros(sym[0].size, dtype=np.uint32) for _ in range(need)]
        timed("recover_data", lambda: rs.RecoverData(sym, have, rec))
        row["verified"] = bool(np.array_equal(o, data))
        out[f"{kib}k"] = row
    print(json.dumps(out))


if __name__ == "__main__":
    main()
