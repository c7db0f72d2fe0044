#!/usr/bin/env python3
"""Sweep the proxy-level load (tools/proxy_load.cpp, bench.py host_path.pooled)
over concurrent request counts and object sizes, one JSON line per point.

    python tools/proxy_sweep.py --threads 1,4,8,16,25 --mib 64,1 --pattern 0 --seconds 1.5

Environment knobs of the library (SLIME_RS_COPY_THREADS, ...) apply as set for
the process.  Tools only: the product's measurement is bench.py's leg."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,4,8,16,25")
    ap.add_argument("--mib", default="64,1")
    ap.add_argument("--pattern", type=int, default=0, help="0 fused entry points, 1 the unchanged Go caller")
    ap.add_argument("--seconds", type=float, default=1.5)
    ap.add_argument("--need", type=int, default=8)
    ap.add_argument("--total", type=int, default=12)
    ap.add_argument("--sched", choices=["auto", "spin", "yield", "blocking"], default="auto",
                    help="hipSetDeviceFlags on every device before the sweep (how host threads wait for the GPU)")
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime per process: torch's)
    from slime_amd import _native as N
    if a.sched != "auto":
        # the HIP runtime already in the process (torch's), by soname
        hip = ctypes.CDLL("libamdhip64.so.7", mode=os.RTLD_NOLOAD | os.RTLD_GLOBAL)
        flag = {"spin": 1, "yield": 2, "blocking": 4}[a.sched]
        for d in range(N.lib.slime_rs_device_count()):
            torch.cuda.set_device(d)
            torch.cuda.synchronize()
            rc = hip.hipSetDeviceFlags(ctypes.c_uint(flag))
            print(json.dumps({"hipSetDeviceFlags": a.sched, "device": d, "rc": rc}), flush=True)
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libproxy_load.so"))
    lib.proxy_load.restype = ctypes.c_int
    lib.proxy_load.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                               ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_double, ctypes.c_uint64,
                               ctypes.POINTER(ctypes.c_double)]
    erase = list(range(a.total - a.need))
    have = [i for i in range(a.total) if i not in erase][:a.need]
    c_have = (ctypes.c_int * a.need)(*have)
    ndev = N.lib.slime_rs_device_count()
    for mib in [int(x) for x in a.mib.split(",")]:
        for t in [int(x) for x in a.threads.split(",")]:
            before = [N.pool_calls(d)[0] for d in range(ndev)]
            out = (ctypes.c_double * 10)()
            rc = lib.proxy_load(t, mib << 20, a.need, a.total, c_have, a.pattern, a.seconds, 0x77 + t, out)
            after = [N.pool_calls(d)[0] for d in range(ndev)]
            wall = out[1] or 1e-9
            print(json.dumps({"threads": t, "object_mib": mib, "pattern": a.pattern, "sched": a.sched,
                              "copy_threads_env": os.environ.get("SLIME_RS_COPY_THREADS"),
                              "gibs": round(2 * out[0] * (mib << 20) / 2**30 / wall, 2),
                              "requests_per_s": round(out[0] / wall, 1),
                              "put_ms": [round(out[4], 3), round(out[5], 3)], "get_ms": [round(out[6], 3), round(out[7], 3)],
                              "per_device_calls": [x - y for x, y in zip(after, before)],
                              "verified": rc == 0 and out[2] == 1.0, "status": rc}), flush=True)


if __name__ == "__main__":
    main()
