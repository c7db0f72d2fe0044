"""Timeline of one host call from a rocprofv3 kernel + HIP-API trace.

Usage: python tools/call_timeline.py <dir with *_kernel_trace.csv and *_hip_api_trace.csv> [call_index] [sync_fn]

Calls are cut at each completed `sync_fn` (default hipEventSynchronize) on the
calling thread; prints call `call_index`'s HIP API calls and kernels (name,
start and end in us from the call's first API entry), then the median call
split over every call of the same shape: API time on the host, first kernel
start, last kernel end, sync return.
"""
import csv
import glob
import os
import statistics
import sys


def rows(d, suffix):
    f = glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True)
    assert f, f"no *{suffix} under {d}"
    with open(f[0]) as fh:
        return list(csv.DictReader(fh))


def main():
    d = sys.argv[1]
    want = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    sync = sys.argv[3] if len(sys.argv) > 3 else "hipEventSynchronize"
    api = rows(d, "hip_api_trace.csv")
    ker = rows(d, "kernel_trace.csv")
    api = [(int(a["Start_Timestamp"]), int(a["End_Timestamp"]), a["Function"], a["Thread_Id"]) for a in api]
    ker = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Kernel_Name"]) for k in ker]
    api.sort()
    ker.sort()
    main_tid = api[0][3]
    api = [a for a in api if a[3] == main_tid]
    calls, cur = [], []
    for a in api:
        cur.append(a)
        if a[2] == sync:
            calls.append(cur)
            cur = []
    print(f"{len(calls)} calls cut at {sync}")
    if want >= len(calls):
        return
    c = calls[want]
    t0 = c[0][0]
    t1 = c[-1][1]
    for s, e, f, _ in c:
        print(f"  api {f:32s} {(s - t0) / 1e3:8.2f} {(e - t0) / 1e3:8.2f}")
    for s, e, n in ker:
        if t0 <= s <= t1:
            print(f"  ker {n[:60]:60s} {(s - t0) / 1e3:8.2f} {(e - t0) / 1e3:8.2f}")
    # Median split over calls with the same API sequence as call `want`.
    sig = [f for _, _, f, _ in c]
    split = []
    for cc in calls:
        if [f for _, _, f, _ in cc] != sig:
            continue
        a0, a1 = cc[0][0], cc[-1][1]
        ks = [k for k in ker if a0 <= k[0] <= a1]
        if not ks:
            continue
        split.append(((cc[-1][0] - a0) / 1e3, (ks[0][0] - a0) / 1e3, (ks[-1][1] - a0) / 1e3, (a1 - a0) / 1e3,
                      sum(k[1] - k[0] for k in ks) / 1e3))
    if split:
        med = [statistics.median(x) for x in zip(*split)]
        print(f"{len(split)} calls like it, median us: sync entered {med[0]:.2f}, first kernel start {med[1]:.2f}, "
              f"last kernel end {med[2]:.2f}, sync returned {med[3]:.2f}, kernel busy {med[4]:.2f}")


if __name__ == "__main__":
    main()
