#!/usr/bin/env python3
"""Concurrent callers of the object entry points, as a slime proxy issues them
(up to 25 HTTP goroutines, main.go:107-109, plus scrubbers, multi.go:54-58):
T threads, each writing (or reconstructing) its own 64 MiB 8/12 objects back
to back; aggregate object GiB/s over the wall time, per T.  ctypes releases
the GIL for the C calls, so the threads run the library concurrently.

    python tools/host_concurrency.py [--threads 1,2,4,8,16] [--reps 6] [--mib 64 | --kib 4]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GIB = float(1 << 30)


def throttled_usec() -> int:
    """CPU time the cgroup's quota withheld so far (cpu.stat throttled_usec; 0 if unreadable)."""
    try:
        for line in open("/sys/fs/cgroup/cpu.stat"):
            k, v = line.split()
            if k == "throttled_usec":
                return int(v)
    except (OSError, ValueError):
        pass
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,2,4,8,16")
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--kib", type=int, default=0, help="object size in KiB (overrides --mib): small-object calls")
    ap.add_argument("--need", type=int, default=8)
    ap.add_argument("--total", type=int, default=12)
    ap.add_argument("--delay", type=float, default=15.0,
                    help="seconds to wait first: a fresh box may still be wiping VRAM an earlier job freed, "
                         "which slows every DMA (DESIGN.md End-to-end)")
    args = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (one HIP runtime: torch first)
    from slime_amd import objects
    need, total = args.need, args.total
    tmax = max(int(t) for t in args.threads.split(","))
    size = (args.kib << 10) if args.kib else (args.mib << 20)
    cb = objects.chunk_size(size, need)
    rng = np.random.default_rng(25)
    objs = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(tmax)]
    chunks = [[np.zeros(cb, dtype=np.uint8) for _ in range(total)] for _ in range(tmax)]
    outs = [np.zeros(size, dtype=np.uint8) for _ in range(tmax)]
    maps = [0] * tmax
    for i in range(tmax):  # warm every buffer and every thread's first call
        maps[i] = objects.write_chunks(objs[i], need, total, out=chunks[i])[0]
    have = list(range(total - need, total))
    results = []
    t_end = time.time() + args.delay
    while time.time() < t_end:  # a single-caller probe every ~2 s while waiting
        t0 = time.perf_counter()
        objects.write_chunks(objs[0], need, total, out=chunks[0])
        print(json.dumps({"probe_write_gibs": round(size / GIB / (time.perf_counter() - t0), 2)}), flush=True)
        time.sleep(2)

    def run(kind: str, T: int) -> float:
        errors = []
        go = threading.Barrier(T + 1)

        def work(i):
            try:
                go.wait()
                for _ in range(args.reps):
                    if kind == "write":
                        objects.write_chunks(objs[i], need, total, out=chunks[i])
                    elif kind == "write_zero_copy":
                        objects.write_chunks(objs[i], need, total, out=chunks[i], alias=True)
                    elif kind == "write_digest":
                        objects.write_chunks_digest(objs[i], need, total, out=chunks[i])
                    else:
                        objects.reconstruct([chunks[i][j] for j in have], have, maps[i], size, out=outs[i])
            except Exception as e:  # noqa: BLE001 - reported below
                errors.append(repr(e))

        th = [threading.Thread(target=work, args=(i,)) for i in range(T)]
        for t in th:
            t.start()
        go.wait()
        t0 = time.perf_counter()
        for t in th:
            t.join()
        dt = time.perf_counter() - t0
        assert not errors, errors
        return T * args.reps * size / GIB / dt, T * args.reps / dt

    for kind in ("write", "write_zero_copy", "reconstruct", "write_digest"):
        for T in (int(t) for t in args.threads.split(",")):
            time.sleep(0.5)  # let the cgroup's CPU quota refill between runs
            th0 = throttled_usec()
            g, calls = run(kind, T)
            results.append({"kind": kind, "threads": T, "gibs": round(g, 2), "calls_per_s": round(calls),
                            "throttled_ms": round((throttled_usec() - th0) / 1e3, 1)})
            print(json.dumps(results[-1]), flush=True)
    ok = all(outs[i].tobytes() == objs[i].tobytes() for i in range(tmax))
    print(json.dumps({"verified": ok, "object_bytes": size, "code": f"{need}/{total}", "reps": args.reps}))


if __name__ == "__main__":
    main()
