#!/usr/bin/env python3
"""End-to-end rate of the Go-API entry points on host (pageable numpy)
buffers: CreateParities and RecoverData at need=8/total=12, PCIe-inclusive.
Compares the staged pipeline (pinned ring + copy pool, default) with the
one-shot pageable path (SLIME_RS_HOST_PIPE=direct) and copy-pool sizes, and
reports the raw host<->device link rates for context.

    python tools/host_pipe.py            # all modes (each in a child process)
    python tools/host_pipe.py --one      # current env only, one JSON line
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)


def link_rates():
    import torch
    n = 256 << 20
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    pageable = torch.empty(n, dtype=torch.uint8)
    pageable.fill_(1)
    pinned = torch.empty(n, dtype=torch.uint8).pin_memory()
    out = {}
    for name, fn in (("h2d_pageable", lambda: dev.copy_(pageable)), ("h2d_pinned", lambda: dev.copy_(pinned)),
                     ("d2h_pageable", lambda: pageable.copy_(dev)), ("d2h_pinned", lambda: pinned.copy_(dev))):
        fn()
        torch.cuda.synchronize()
        t = []
        for _ in range(5):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            t.append(time.perf_counter() - t0)
        out[name + "_GBps"] = round(n / statistics.median(t) / 1e9, 1)
    return out


def one(sizes_mib, reps):
    import numpy as np
    from slime_amd import rs
    need, total = 8, 12
    res = {"mode": os.environ.get("SLIME_RS_HOST_PIPE", "staged"),
           "copy_threads": os.environ.get("SLIME_RS_COPY_THREADS", "4"),
           "nt": os.environ.get("SLIME_RS_COPY_NT", "1")}
    rng = np.random.default_rng(1)
    for mib in sizes_mib:
        L = (mib << 20) // (4 * need)
        data = [rng.integers(0, 2**32 - 5, size=L, dtype=np.uint64).astype(np.uint32) for _ in range(need)]
        outs = [np.zeros(L, dtype=np.uint32) for _ in range(total - need)]
        recs = [np.zeros(L, dtype=np.uint32) for _ in range(need)]

        def med(fn):
            fn()
            t = []
            for _ in range(reps):
                t0 = time.perf_counter()
                fn()
                t.append(time.perf_counter() - t0)
            return statistics.median(t)

        enc_fresh = med(lambda: rs.CreateParities(data, total))  # fresh np.zeros rows, as Go's make()
        enc = med(lambda: rs.CreateParities(data, total, outs))  # caller-reused rows
        code = data + outs
        have = list(range(4, 12))
        chunks = [code[i] for i in have]
        dec = med(lambda: rs.RecoverData(chunks, have, recs))
        assert all(np.array_equal(a, b) for a, b in zip(recs, data))
        obj = need * L * 4
        res[f"{mib}MiB"] = {"encode_GiBps": round(obj / enc / GIB, 2),
                            "encode_fresh_out_GiBps": round(obj / enc_fresh / GIB, 2),
                            "recover_GiBps": round(obj / dec / GIB, 2)}
        # object entry points: writeChunks / reconstruct data paths (bytes in, bytes out)
        from slime_amd import objects
        raw = rng.integers(0, 256, size=mib << 20, dtype=np.uint8).tobytes()
        box = {}

        cbufs = [np.zeros(objects.chunk_size(len(raw), need), dtype=np.uint8) for _ in range(total)]
        obuf = np.zeros(len(raw), dtype=np.uint8)

        def wc():
            box["w"] = objects.write_chunks(raw, need, total, out=cbufs)
        wct = med(wc)  # caller-reused chunk buffers (steady state of a store's buffer pool)
        m, chunks = box["w"]
        surv = [chunks[i] for i in have]
        rct = med(lambda: objects.reconstruct(surv, have, m, len(raw), out=obuf))
        assert obuf.tobytes() == raw
        res[f"{mib}MiB"].update({"write_chunks_GiBps": round(len(raw) / wct / GIB, 2),
                                 "reconstruct_GiBps": round(len(raw) / rct / GIB, 2), "mapping": m})
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--one", action="store_true")
    ap.add_argument("--links", action="store_true")
    ap.add_argument("--sizes", default="1,16,64,256")
    ap.add_argument("--reps", type=int, default=7)
    args = ap.parse_args()
    sizes = [int(s) for s in args.sizes.split(",")]
    if args.one:
        print(json.dumps(one(sizes, args.reps)), flush=True)
        return
    if args.links:
        print(json.dumps({"links": link_rates()}), flush=True)
        return
    # The parent never touches the GPU: every measurement runs in a child.
    r = subprocess.run([sys.executable, __file__, "--links"], capture_output=True, text=True, timeout=300)
    print(r.stdout.strip() or json.dumps({"links_rc": r.returncode, "err": r.stderr[-800:]}), flush=True)
    variants = [{"SLIME_RS_HOST_PIPE": "direct"}, {"SLIME_RS_HOST_PIPE": "register"}, {"SLIME_RS_COPY_THREADS": "0"}, {"SLIME_RS_COPY_THREADS": "2"},
                {}, {"SLIME_RS_COPY_THREADS": "8"}, {"SLIME_RS_COPY_NT": "0"},
                {"SLIME_RS_PIPE_TRACE": "1", "SLIME_RS_COPY_THREADS": "4"}]
    for v in variants:
        env = dict(os.environ, **v)
        r = subprocess.run([sys.executable, __file__, "--one", "--sizes", args.sizes, "--reps", str(args.reps)],
                           env=env, capture_output=True, text=True, timeout=300)
        print(r.stdout.strip() or json.dumps({"variant": v, "rc": r.returncode, "err": r.stderr[-800:]}), flush=True)
        if "SLIME_RS_PIPE_TRACE" in v:  # per-call host-time split, last call of each size
            lines = [ln for ln in r.stderr.splitlines() if ln.startswith("slime_rs ")]
            seen = {}
            for ln in lines:
                seen[" ".join(ln.split()[1:3])] = ln
            for ln in seen.values():
                print("  " + ln, flush=True)


if __name__ == "__main__":
    main()
