#!/usr/bin/env python3
"""Where a dynamic-schedule apply launch's fixed cost goes.

C2 (4/6, 64 MiB objects) fits 25 us fixed + 17 us per object across batches of
32 / 64 / 128 objects (profiles/r05/s4_pmc_c2/).  This runs, in one process on
one buffer from the bench's allocator, for each batch size:

  - the product encode launch (the library; HIP events between launches
    enqueued back to back, as the bench times them), and
  - its stamped twin (tools/c2_stamps.hip: the same kernel template, geometry,
    spread and block count, STAMP = 2), whose waves record s_memrealtime
    (100 MHz) at start, first loads issued, tiles 4 / 16 / 64, last stores
    issued, stores retired, and exit counted,

checks the twin's output against the product's, and splits one launch into:

  between     event interval - (last wave's exit - first wave's start), launches
              back to back: the end of one kernel and the dispatch of the next
  ramp        first wave start -> last wave start, and each wave's setup (start
              -> first loads issued: its first ticket's round trip); then each
              wave's per-tile time over its tiles 0-4, 4-16, 16-64 against its
              steady rate past tile 64 (early_excess: the slow start)
  drain       first wave to find the queue dry (stores issued) -> last wave's
              stores retired: the imbalance tail
  reset       the last-out wave's exit count + counter reset (finish)
and fits event time and wave span against the object count (a + b * nobj).

    make tools/libc2stamps.so && python tools/c2_stamps.py [--need 4 --total 6 --mib 64 --nobj 32,64,128]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from slime_amd import device as D  # noqa: E402

TICK_US = 0.01  # s_memrealtime: 100 MHz


def fit(xs, ys):
    b, a = np.polyfit(np.asarray(xs, float), np.asarray(ys, float), 1)
    return {"fixed_us": round(a, 2), "per_object_us": round(b, 3)}


def analyse(rec: np.ndarray, event_ms: float) -> dict:
    t0, tw, t4, t16, t64, ti, tr, te = (rec[:, i].astype(np.float64) for i in range(8))
    meta = rec[:, 8].astype(np.uint64)
    tiles = ((meta >> np.uint64(32)) & np.uint64(0x7FFFFFFF)).astype(np.int64)
    last = (meta >> np.uint64(63)).astype(bool)
    base = t0.min()
    us = lambda v: round(float(v) * TICK_US, 2)  # noqa: E731
    span = te.max() - base
    last_i = int(np.argmax(last)) if last.any() else int(np.argmax(te))
    first_dry = ti.min()
    # Per-tile time of each phase of a wave's walk (waves that reached tile 64
    # and walked past it): the steady rate is the last phase's.
    ok = (t64 > 0) & (tiles > 64)
    steady = np.median((ti[ok] - t64[ok]) / (tiles[ok] - 64))
    ph = {"start_to_tile4": (t4[ok] - t0[ok], 4), "tile4_to_16": (t16[ok] - t4[ok], 12),
          "tile16_to_64": (t64[ok] - t16[ok], 48)}
    phases = {k: {"per_tile_us": us(np.median(d) / n), "excess_us": us(np.median(d) - n * steady)}
              for k, (d, n) in ph.items()}
    out = {
        "waves": int(len(t0)), "event_us": round(event_ms * 1e3, 2), "wave_span_us": us(span),
        "between_waves_us": round(event_ms * 1e3 - span * TICK_US, 2),
        "ramp": {"start_spread_us": us(t0.max() - base),
                 "setup_us": {"p50": us(np.median(tw - t0)), "p90": us(np.percentile(tw - t0, 90)),
                              "max": us((tw - t0).max())}},
        "steady_tile_us": us(steady), "early_phases": phases,
        "early_excess_us": round(sum(v["excess_us"] for v in phases.values()), 2),
        "walk_end_us": {q: us(np.percentile(ti - base, p)) for q, p in (("first", 0), ("p50", 50), ("max", 100))},
        "drain": {"first_dry_to_last_retired_us": us(tr.max() - first_dry),
                  "p50_issued_to_last_retired_us": us(tr.max() - np.median(ti)),
                  "retire_wait_us": {"p50": us(np.median(tr - ti)), "max": us((tr - ti).max())}},
        "reset": {"exit_count_us_p50": us(np.median(te - tr)), "last_out_exit_us": us(te[last_i] - tr[last_i]),
                  "last_out_is_last_to_end": bool(te[last_i] >= te.max() - 1)},
        "tiles_per_wave": [int(tiles.min()), int(np.median(tiles)), int(tiles.max())],
    }
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--need", type=int, default=4)
    ap.add_argument("--total", type=int, default=6)
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--nobj", type=str, default="32,64,128")
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--geometry", type=str, default="0:0",
                    help="stamped twin geometries spread:blocks[:kcode] (0 = the product's rule; kcode selects a "
                         "unroll/unit variant of tools/c2_stamps.hip, default need), comma list; the split is "
                         "reported for the first")
    args = ap.parse_args()
    need, total = args.need, args.total
    r = total - need
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libc2stamps.so"))
    lib.cs_launch.restype = ctypes.c_int
    lib.cs_launch.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_uint64] * 4 + [ctypes.c_void_p] * 3 + \
        [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32, ctypes.c_uint32]
    L = -(-(args.mib << 20) // 4 // need)
    SS = -(-L // 64) * 64  # the bench's line-aligned shard stride
    counts = [int(x) for x in args.nobj.split(",")]
    nmax = max(counts)
    buf = D.device_empty(nmax * total * SS, torch.int32, 0)
    D.fill_symbols(buf, 0x5113E)
    enc = D.Plan.encode(need, total)
    lay = D.layout_of(total, L, SS)
    coeff = np.zeros((r, max(16, -(-need // 16) * 16)), dtype=np.uint32)
    coeff[:, :need] = enc.coefficients()
    c_t = torch.from_numpy(coeff.view(np.int32).reshape(-1)).cuda()
    ii = torch.arange(need, dtype=torch.int32, device="cuda")
    oi = torch.arange(need, total, dtype=torch.int32, device="cuda")
    ticket = torch.zeros(64 * 64, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    res = {"shape": f"{need}/{total} {args.mib} MiB", "L": L, "shard_stride": SS, "batches": {}}
    ev_fit, span_fit = [], []
    for nobj in counts:
        b = buf[: nobj * total * SS]
        par = lambda: b.view(nobj, total, SS)[:, need:, :L]  # noqa: E731

        def product():
            enc(b, lay, b, lay, L, nobj, stream=s, dst_offset=need * SS)

        nw = ctypes.c_uint32(0)
        geos = [tuple(int(v) for v in (g + ":" + str(need) if g.count(":") == 1 else g).split(":"))
                for g in args.geometry.split(",")]
        nws = {}
        for g in geos:
            rc = lib.cs_launch(g[2], b.data_ptr(), b.data_ptr(), total * SS, SS, total * SS, SS, c_t.data_ptr(),
                               ii.data_ptr(), oi.data_ptr(), L, nobj, r, ctypes.c_void_p(s.cuda_stream),
                               ticket.data_ptr(), None, ctypes.byref(nw), g[0], g[1])
            assert rc == 0, rc
            nws[g] = nw.value
        st = torch.zeros(max(nws.values()) * 9, dtype=torch.int64, device="cuda")

        def stamped_at(g):
            def fn():
                rc = lib.cs_launch(g[2], b.data_ptr(), b.data_ptr(), total * SS, SS, total * SS, SS, c_t.data_ptr(),
                                   ii.data_ptr(), oi.data_ptr(), L, nobj, r, ctypes.c_void_p(s.cuda_stream),
                                   ticket.data_ptr(), st.data_ptr(), ctypes.byref(nw), g[0], g[1])
                assert rc == 0, rc
            return fn
        stamped = stamped_at(geos[0])

        product()
        torch.cuda.synchronize()
        want = par().clone()
        # Back to back, as the bench's timed loop runs them: events between
        # launches enqueued without a host wait, so an interval is GPU time
        # from one launch's start to the next's (the gap between kernels
        # included), never the host's enqueue latency.
        times, recs, good = {}, [], True
        runs = [("product", product), ("stamped", stamped)] + \
            [(f"stamped_{g[0]}:{g[1]}:{g[2]}", stamped_at(g)) for g in geos[1:]] + [("product2", product)]
        for name, fn in runs:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.reps + 1)]
            ev[0].record(s)
            for i in range(args.reps):
                fn()
                ev[i + 1].record(s)
            torch.cuda.synchronize()
            good = good and bool(torch.equal(par(), want))  # every variant writes the product's parity
            par().zero_()
            times[name] = [ev[i].elapsed_time(ev[i + 1]) for i in range(1, args.reps)]  # the first one warms
            if name == "stamped":
                recs.append((times[name][-1], st.view(-1, 9)[: nws[geos[0]]].cpu().numpy().copy()))
        times["product"] += times.pop("product2")
        ok = good
        med = {k: statistics.median(v) for k, v in times.items()}
        # the stamped launch nearest its median time
        ms, rec = recs[0]  # the last stamped launch of its back-to-back run
        a = analyse(rec, ms)
        alg = nobj * 4 * L * total
        res["batches"][str(nobj)] = {
            "product_ms": round(med["product"], 4), "stamped_ms": round(med["stamped"], 4),
            "product_frac": round(alg / (med["product"] * 1e-3) / 8e12, 4), "stamped_matches_product": ok,
            "geometries": {k: {"ms": round(v, 4), "frac": round(alg / (v * 1e-3) / 8e12, 4)}
                           for k, v in med.items() if k.startswith("stamped")},
            "split": a}
        ev_fit.append(med["product"] * 1e3)
        span_fit.append(a["wave_span_us"])
    res["fit_product_event"] = fit(counts, ev_fit)
    res["fit_stamped_wave_span"] = fit(counts, span_fit)
    print(json.dumps(res, indent=1))
    if not all(v["stamped_matches_product"] for v in res["batches"].values()):
        sys.exit(3)


if __name__ == "__main__":
    main()
