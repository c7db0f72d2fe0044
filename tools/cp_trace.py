"""The unchanged caller's CreateParity x r on one 64 MiB 8/12 object, with the
host pipeline's per-call split (SLIME_RS_PIPE_TRACE=1 prints one line per call
to stderr), tools only.

    SLIME_RS_PIPE_TRACE=1 python tools/cp_trace.py [--mib 64] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from slime_amd import _native as N  # noqa: E402
from slime_amd import gf, objects, rs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--need", type=int, default=8)
    ap.add_argument("--total", type=int, default=12)
    a = ap.parse_args()
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, size=a.mib << 20, dtype=np.uint8)
    _, words = gf.MapToGF(data)
    parts = objects.split_vector(words, a.need)
    r = a.total - a.need
    par = [np.zeros(parts[0].size, dtype=np.uint32) for _ in range(r)]
    for i in range(r):  # warm
        rs.CreateParity(parts, a.need + i, par[i])
    out = []
    for rep in range(a.reps):
        N.host_stats(reset=True)
        t0 = time.perf_counter()
        for i in range(r):
            rs.CreateParity(parts, a.need + i, par[i])
        dt = time.perf_counter() - t0
        st = N.host_stats(reset=True)
        out.append({"rep": rep, "ms_x_r": round(dt * 1e3, 3), "per_call_ms": round(dt * 1e3 / r, 3),
                    "split_us_per_call": {k: round(st[k] / max(1, st["calls"]), 1)
                                          for k in ("copy_in_us", "enqueue_us", "wait_us", "copy_out_us", "total_us")},
                    "windows_per_call": st["windows"] / max(1, st["calls"])})
    print(json.dumps({"object_mib": a.mib, "code": f"{a.need}/{a.total}", "runs": out}))


if __name__ == "__main__":
    main()
