#!/usr/bin/env python3
"""Why do the object entry points run at 10-12 GiB/s in some processes and
25-30 in others, with the same code?  Per process (child), for a copy-pool
size: write_chunks and reconstruct of one 64 MiB 8/12 object, median of
`--reps`, with SLIME_RS_PIPE_TRACE's split of each call (host copy in,
enqueue, event wait, host copy out), the cgroup's CPU-throttling counters
around the timed calls, and the pinned DMA and host memcpy rates measured in
the same process.

    python tools/host_diag.py [--threads 0,2,4,8] [--reps 7]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GIB = float(1 << 30)


def cpu_stat() -> dict:
    try:
        return {k: int(v) for k, v in (line.split() for line in open("/sys/fs/cgroup/cpu.stat"))}
    except (OSError, ValueError):
        return {}


def thread_affinity() -> dict:
    """Cpus_allowed_list of every thread of this process -> thread count."""
    out: dict = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            for line in open(f"/proc/self/task/{tid}/status"):
                if line.startswith("Cpus_allowed_list:"):
                    k = line.split(":", 1)[1].strip()
                    out[k] = out.get(k, 0) + 1
        except OSError:
            pass
    return out


def child(reps: int, pre: str) -> None:
    import numpy as np
    import torch  # noqa: F401  (one HIP runtime: torch first)
    from slime_amd import objects
    aff0 = thread_affinity()
    if pre == "bench":  # what bench.py does before its host leg: device-resident work
        import bench
        from slime_amd import device as D
        buf = torch.empty(1 << 28, dtype=torch.int32, device="cuda")
        D.fill_symbols(buf, 7)
        torch.cuda.synchronize()
        del buf
        _ = bench.board_info(0)
    need, total, S = 8, 12, 64 << 20
    rng = np.random.default_rng(1)
    data = rng.integers(0, 256, size=S, dtype=np.uint8)
    cb = objects.chunk_size(S, need)
    chunks = [np.zeros(cb, dtype=np.uint8) for _ in range(total)]
    out = np.zeros(S, dtype=np.uint8)
    have = list(range(4, 12))
    m = objects.write_chunks(data, need, total, out=chunks)[0]
    surv = [chunks[i] for i in have]
    objects.reconstruct(surv, have, m, S, out=out)
    res = {"pid": os.getpid(), "cpu": os.sched_getaffinity(0).__len__(), "pre": pre,
           "threads_affinity_at_start": aff0}
    for name, fn in (("write_chunks", lambda: objects.write_chunks(data, need, total, out=chunks)),
                     ("reconstruct", lambda: objects.reconstruct(surv, have, m, S, out=out))):
        st0 = cpu_stat()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        st1 = cpu_stat()
        res[name] = {"gibs_median": round(S / GIB / statistics.median(ts), 2),
                     "gibs_best": round(S / GIB / min(ts), 2),
                     "throttled_periods": st1.get("nr_throttled", 0) - st0.get("nr_throttled", 0),
                     "throttled_ms": round((st1.get("throttled_usec", 0) - st0.get("throttled_usec", 0)) / 1e3, 1)}
    assert bytes(out) == data.tobytes()
    res["threads_affinity_after"] = thread_affinity()
    print("RESULT " + json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="0,2,4,8")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--pre", default="none", help="none | bench: run bench.py's device-resident steps first")
    a = ap.parse_args()
    if a.child:
        child(a.reps, a.pre)
        return
    rows = []
    for t in a.threads.split(","):
        env = dict(os.environ, SLIME_RS_COPY_THREADS=t, SLIME_RS_PIPE_TRACE="1")
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--reps", str(a.reps), "--pre", a.pre],
                           capture_output=True, text=True, timeout=600, env=env)
        if r.returncode != 0:
            print(r.stdout[-2000:], r.stderr[-3000:], file=sys.stderr)
            sys.exit(r.returncode)
        res = json.loads(next(line for line in r.stdout.splitlines() if line.startswith("RESULT "))[7:])
        split = {}
        for what in ("write_chunks", "reconstruct"):
            vals = [tuple(float(x) for x in m) for m in re.findall(
                what + r" windows=\d+ copy_in=([\d.]+) enqueue=([\d.]+) wait=([\d.]+) copy_out=([\d.]+) total=([\d.]+)",
                r.stderr)]
            if vals:
                cols = list(zip(*vals))
                split[what] = {k: round(statistics.median(c), 3) for k, c in
                               zip(("copy_in_ms", "enqueue_ms", "wait_ms", "copy_out_ms", "total_ms"), cols)}
        res["copy_threads"] = int(t)
        res["trace_median"] = split
        rows.append(res)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
