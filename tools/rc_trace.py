"""Fused reconstruct of one 64 MiB 8/12 object from host memory, a few calls
back to back (for rocprofv3 --kernel-trace --memory-copy-trace: do the
copy engines' uploads overlap the kernel downloads?), tools only.

    python tools/rc_trace.py [--mib 64] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from slime_amd import objects  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    need, total = 8, 12
    data = np.random.default_rng(3).integers(0, 256, size=a.mib << 20, dtype=np.uint8)
    cb = objects.chunk_size(data.size, need)
    chunks = [np.zeros(cb, dtype=np.uint8) for _ in range(total)]
    m, _ = objects.write_chunks(data, need, total, out=chunks)
    have = list(range(4, 12))
    surv = [chunks[i] for i in have]
    out = np.zeros(data.size, dtype=np.uint8)
    objects.reconstruct(surv, have, m, data.size, out=out)
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        objects.reconstruct(surv, have, m, data.size, out=out)
        ts.append(round((time.perf_counter() - t0) * 1e3, 3))
    print(json.dumps({"reconstruct_ms": ts, "verified": bool(np.array_equal(out, data))}))


if __name__ == "__main__":
    main()
