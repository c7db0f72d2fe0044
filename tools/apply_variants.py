#!/usr/bin/env python3
"""A/B the apply-kernel variants (tools/apply_variants.hip) on the C3/C4 shape.

Variants: U (16-byte units per lane per step: 1 or 2, the wave streaming 1 or
2 KiB of every shard), nt loads, nt stores; geometries: total resident blocks
x objects in flight.  Interleaved rounds in one process (cdna guide rule 24);
every variant's output is checked bit-exact against the product kernel.

    make applyvar && python tools/apply_variants.py [--need 8 --total 12 --mib 256 --nobj 128]
"""
from __future__ import annotations

import argparse
import ctypes
import itertools
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from slime_amd import device as D  # noqa: E402

BATCHED: dict = {}  # variant id -> U
QUEUE: dict = {}  # variant id -> tiles per wave unit (C)
BURST: dict = {}  # variant id -> tiles per store burst
PHASED: dict = {}  # variant id -> (U, period ticks, read-window ticks)
ALL_VARIANTS = {0: "U1 ntL", 1: "U1 plain", 2: "U1 ntL ntS", 3: "U1 ntS", 4: "U2 ntL", 5: "U2 plain",
                6: "U2 ntL ntS", 7: "U2 ntS", 8: "U4 ntL ntS", 9: "U4 ntL", 10: "U3 ntL ntS",
                11: "U4 ntL ntS rot", 12: "U2 ntL ntS rot",
                13: "pipe U1 ntL ntS", 14: "pipe U2 ntL ntS", 15: "pipe U3 ntL ntS",
                16: "pipe U3 XOR-math (wrong by design)", 17: "pipe U2 XOR-math (wrong by design)",
                18: "pipe U3 read-only probe", 19: "pipe U3 write-only probe", 20: "pipe U4 ntL ntS", 21: "pipe U3 XCD-grouped"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--need", type=int, default=8)
    ap.add_argument("--total", type=int, default=12)
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--nobj", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", type=str, default="0,2,4,6,8,9,10")
    ap.add_argument("--blocks", type=str, default="256,384,512,768,1024")
    ap.add_argument("--inflight", type=str, default="0", help="work items (object segments) in flight (0 = all)")
    ap.add_argument("--nseg", type=str, default="1", help="column segments per object (comma list)")
    ap.add_argument("--decode", type=int, default=0, help="time reconstruct of data 0..e-1 instead of encode")
    ap.add_argument("--pad", type=str, default="0", help="shard stride = L + pad symbols (comma list)")
    ap.add_argument("--hunt", choices=["any", "slow", "fast"], default="any",
                    help="re-allocate until the product encode runs in the given placement mode")
    ap.add_argument("--phased", type=str, default="",
                    help="time-phased walks U:period:rwin (100 MHz ticks), comma list, e.g. 3:700:460,6:1400:930")
    ap.add_argument("--pipek", type=str, default="", help="k > 16 through the pipelined k-template kernel: U list")
    ap.add_argument("--wide", type=int, default=0, help="k > 16: time the wide kernel with field math (500) and XOR (501)")
    ap.add_argument("--batched", type=str, default="", help="register-batched stores: U list (2,3)")
    ap.add_argument("--queue", type=str, default="",
                    help="dynamic-schedule walk (rs_apply_queue_kernel, U3): C + 100 * NC + 10000 * TB (tiles per wave "
                         "unit, ticket counters, tickets per atomic), comma list, e.g. 104,802,20802")
    ap.add_argument("--burst", type=str, default="", help="LDS-staged write bursts: tiles per burst, comma list (1..3)")
    ap.add_argument("--timed", type=int, default=0,
                    help="also run the product walk with per-wave stamps N times per geometry (k = 8, U = 3): tail report")
    ap.add_argument("--separate", type=int, default=-1,
                    help="1: write to a separate buffer, 0: in place (default: encode in place, decode separate)")
    args = ap.parse_args()
    VARIANTS = {int(v): ALL_VARIANTS[int(v)] for v in args.variants.split(",") if v}
    PHASED.clear()
    for i, spec in enumerate(x for x in args.phased.split(",") if x):
        u, per, rw = (int(t) for t in spec.split(":"))
        assert rw >= 50 and per - rw >= 50, "phase windows must be >= 50 ticks"
        PHASED[100 + i] = (u, per, rw)
        VARIANTS[100 + i] = f"phased U{u} period {per} read {rw} ticks"
    for t in (int(x) for x in args.burst.split(",") if x):
        BURST[200 + t] = t
        VARIANTS[200 + t] = f"pipe U3 + LDS-staged store bursts of {t} tiles"
    if args.wide:
        VARIANTS.clear()
        VARIANTS[500] = "wide pipe, field math (product)"
        VARIANTS[501] = "wide pipe, XOR stand-in (wrong by design)"
    for u in (int(x) for x in args.pipek.split(",") if x):
        VARIANTS[700 + u] = f"pipe K={args.need} U{u} (k-template kernel)"
    for c in (int(x) for x in args.queue.split(",") if x):
        QUEUE[400 + c] = c
        pol = {1: "", 2: " plain stores", 3: " plain loads", 4: " plain loads+stores"}.get(c // 10000000, "")
        VARIANTS[400 + c] = (f"queue U{c // 100000 % 10 or 3} C{c % 100} NC{c // 100 % 100} TB{max(1, c // 10000 % 10)}"
                             f"{' on-demand' if 1000000 <= c < 10000000 else ''}{pol} (dynamic schedule)")
    for u in (int(x) for x in args.batched.split(",") if x):
        BATCHED[300 + u] = u
        VARIANTS[300 + u] = f"pipe U{u} + all rows in registers, stores back to back"
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libapplyvar.so"))
    lib.av_launch_pipek.restype = ctypes.c_int
    lib.av_launch_pipek.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_uint64] * 4 + \
        [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.c_void_p, ctypes.c_uint32]
    lib.av_launch_wide.restype = ctypes.c_int
    lib.av_launch_wide.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_uint64] * 4 + \
        [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
    lib.av_launch_batched.restype = ctypes.c_int
    lib.av_launch_batched.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_uint64] * 4 + \
        [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.c_void_p, ctypes.c_uint32]
    lib.av_launch_burst.restype = ctypes.c_int
    lib.av_launch_burst.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_uint64] * 4 + \
        [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.c_void_p, ctypes.c_uint32]
    lib.av_launch_phased.restype = ctypes.c_int
    lib.av_launch_phased.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_uint64] * 4 + \
        [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
    lib.av_launch_queue.restype = ctypes.c_int
    lib.av_launch_queue.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_uint64] * 4 + \
        [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
    lib.av_launch_timed.restype = ctypes.c_int
    lib.av_launch_timed.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint64] * 4 + [ctypes.c_void_p] * 3 + \
        [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
         ctypes.c_uint32, ctypes.c_void_p]
    lib.av_launch.restype = ctypes.c_int
    lib.av_launch.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_uint64] * 4 + \
        [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
    need, total, nobj = args.need, args.total, args.nobj
    r = total - need
    L = -(-(args.mib << 20) // 4 // need)  # perVector = ceil(ceil(S/4)/need), splitVector
    pads = [int(p) for p in args.pad.split(",")]
    maxss = L + max(pads)
    tail = nobj * r * maxss if args.separate == 2 else 0  # 2: destination in the same allocation, after the objects
    enc = D.Plan.encode(need, total)
    hunt_ms, keep = [], []
    for attempt in range(24):
        whole = torch.empty(nobj * total * maxss + tail, dtype=torch.int32, device="cuda")
        if args.hunt == "any":
            break
        lay0 = D.layout_of(total, L)
        probe = whole[: nobj * total * L]
        D.fill_symbols(probe, 7)
        t = []
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            enc(probe, lay0, probe, lay0, L, nobj, dst_offset=need * L)
            b.record()
            torch.cuda.synchronize()
            t.append(a.elapsed_time(b))
        hunt_ms.append(round(min(t[1:]), 3))
        slow = min(t[1:]) > 9.2 * (nobj / 128) * (args.mib / 256)
        if (args.hunt == "slow") == slow:
            break
        keep = (keep + [whole])[-2:]  # hold the last two so the next allocation lands elsewhere
        torch.cuda.empty_cache()
    del keep
    torch.cuda.empty_cache()
    results_by_pad = {}
    for pad in pads:
        results_by_pad[pad] = run_pad(args, lib, whole, enc, need, total, r, nobj, L, L + pad, VARIANTS)
    print(json.dumps({"shape": f"{need}/{total} {args.mib} MiB x {nobj}", "decode": bool(args.decode),
                      "hunt": args.hunt, "hunt_probe_ms": hunt_ms, "by_pad": results_by_pad}, indent=1))


def run_pad(args, lib, whole, enc, need, total, r, nobj, L, SS, VARIANTS):
    buf = whole[: nobj * total * SS]
    D.fill_symbols(buf, 7)
    lay = D.layout_of(total, L, SS)
    enc(buf, lay, buf, lay, L, nobj, dst_offset=need * SS)
    torch.cuda.synchronize()
    shards = lambda: buf.view(nobj, total, SS)[:, :, :L]  # noqa: E731
    ref = shards()[:, need:, :].clone()

    coeff = np.zeros((r, max(16, -(-need // 16) * 16)), dtype=np.uint32)
    s = torch.cuda.current_stream()
    separate = args.separate if args.separate >= 0 else int(bool(args.decode))
    if args.decode:
        # Rebuild data shards 0..r-1 from shards r..total-1.
        have = list(range(r, total))
        dec = D.Plan.reconstruct(need, total, have, list(range(r)))
        coeff[:, :need] = dec.coefficients()
        ii = torch.tensor(have, dtype=torch.int32, device="cuda")
        ref = shards()[:, :r, :].clone()
        slot0 = 0
    else:
        coeff[:, :need] = enc.coefficients()
        ii = torch.arange(need, dtype=torch.int32, device="cuda")
        slot0 = need
    if separate:
        dst = whole[whole.numel() - nobj * r * SS:] if args.separate == 2 else \
            torch.empty(nobj * r * SS, dtype=torch.int32, device="cuda")
        oi = torch.arange(r, dtype=torch.int32, device="cuda")
        d_ptr, oo, view = dst.data_ptr(), r * SS, lambda: dst.view(nobj, r, SS)[:, :, :L]
    else:
        oi = torch.arange(slot0, slot0 + r, dtype=torch.int32, device="cuda")
        d_ptr, oo = buf.data_ptr(), total * SS
        view = lambda: shards()[:, slot0:slot0 + r, :]  # noqa: E731
    c_t = torch.from_numpy(coeff.view(np.int32).reshape(-1)).cuda()
    ticket = torch.zeros(32 * 64, dtype=torch.int32, device="cuda")  # counters + the zero_next set
    stamp_ptr = [None]  # queue variants record per-wave stamps here when set (--timed)

    def launch(v, gx, gy, nseg=1):
        if 700 <= v < 800:
            rc = lib.av_launch_pipek(need, v - 700, buf.data_ptr(), d_ptr, total * SS, SS, oo, SS, c_t.data_ptr(),
                                     ii.data_ptr(), oi.data_ptr(), L, nobj, r, gx, gy, ctypes.c_void_p(s.cuda_stream),
                                     nseg)
            assert rc == 0, rc
            return
        if v in (500, 501):
            rc = lib.av_launch_wide(int(v == 500), buf.data_ptr(), d_ptr, total * SS, SS, oo, SS, c_t.data_ptr(),
                                    ii.data_ptr(), oi.data_ptr(), L, nobj, r, need, gx, gy,
                                    ctypes.c_void_p(s.cuda_stream), nseg)
            assert rc == 0, rc
            return
        if v in QUEUE:
            ticket.zero_()
            rc = lib.av_launch_queue(QUEUE[v], need, buf.data_ptr(), d_ptr, total * SS, SS, oo, SS, c_t.data_ptr(),
                                     ii.data_ptr(), oi.data_ptr(), L, nobj, r, gx * gy,
                                     ctypes.c_void_p(s.cuda_stream), ticket.data_ptr(), stamp_ptr[0], nseg)
            assert rc == 0, rc
            return
        if v in BATCHED:
            assert r == 4 and need == 8, "batched walk is built for 8/12 (4 rows)"
            rc = lib.av_launch_batched(BATCHED[v], buf.data_ptr(), d_ptr, total * SS, SS, oo, SS, c_t.data_ptr(),
                                       ii.data_ptr(), oi.data_ptr(), L, nobj, gx, gy, ctypes.c_void_p(s.cuda_stream),
                                       nseg)
            assert rc == 0, rc
            return
        if v in BURST:
            assert r == 4 and need == 8, "burst walk is built for 8/12 (4 rows)"
            rc = lib.av_launch_burst(BURST[v], buf.data_ptr(), d_ptr, total * SS, SS, oo, SS, c_t.data_ptr(),
                                     ii.data_ptr(), oi.data_ptr(), L, nobj, gx, gy, ctypes.c_void_p(s.cuda_stream),
                                     nseg)
            assert rc == 0, rc
            return
        if v in PHASED:
            assert r == 4 and need == 8, "phased walk is built for 8/12 (4 rows)"
            u, per, rw = PHASED[v]
            rc = lib.av_launch_phased(u, buf.data_ptr(), d_ptr, total * SS, SS, oo, SS, c_t.data_ptr(), ii.data_ptr(),
                                      oi.data_ptr(), L, nobj, gx, gy, ctypes.c_void_p(s.cuda_stream), nseg, per, rw)
            assert rc == 0, rc
            return
        rc = lib.av_launch(v, need, buf.data_ptr(), d_ptr, total * SS, SS, oo, SS, c_t.data_ptr(),
                           ii.data_ptr(), oi.data_ptr(), L, nobj, r, gx, gy, ctypes.c_void_p(s.cuda_stream), nseg)
        assert rc == 0, rc

    segs = [int(x) for x in args.nseg.split(",")]
    geos = []
    for t, y0, ns in itertools.product(args.blocks.split(","), args.inflight.split(","), segs):
        y = nobj * ns if int(y0) == 0 else int(y0)
        if y <= nobj * ns:
            geos.append((int(t), y, ns))
    times = {(v, g): [] for v in VARIANTS for g in geos}
    for _ in range(args.rounds):
        for v in VARIANTS:
            for t, y, ns in geos:
                gx = max(1, t // y)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                launch(v, gx, y, ns)
                b.record(s)
                torch.cuda.synchronize()
                times[(v, (t, y, ns))].append(a.elapsed_time(b))
    # correctness of every variant and segment count
    bad = []
    for v in VARIANTS:
        if v == 501:
            continue  # wrong by design
        for ns in segs:
            view().zero_()
            launch(v, 4, 8, ns)
            torch.cuda.synchronize()
            if not torch.equal(view(), ref):
                bad.append((v, ns))
    alg = nobj * 4 * L * total
    tails = []

    def tail_report(label, geo, ms, rec):
        t0, t1 = rec[:, 0].astype(np.float64), rec[:, 1].astype(np.float64)
        xcc = (rec[:, 2] & 0xFFFFFFFF).astype(np.int64)
        tiles = (rec[:, 2] >> 32).astype(np.int64)
        base = t0.min()
        end = (t1 - base) / 100.0  # 100 MHz ticks -> us
        span = end.max()
        per_xcc = {int(x): {"waves": int((xcc == x).sum()), "end_med_us": round(float(np.median(end[xcc == x])), 1),
                            "end_max_us": round(float(end[xcc == x].max()), 1), "tiles": int(tiles[xcc == x].sum())}
                   for x in sorted(set(xcc.tolist()))}
        t, y, ns = geo
        return {"variant": label, "blocks": t, "objects_in_flight": y, "nseg": ns, "event_ms": round(ms, 3),
                "start_spread_us": round(float((t0.max() - base) / 100.0), 1),
                "end_us": {q: round(float(np.percentile(end, p)), 1)
                           for q, p in (("min", 0), ("p10", 10), ("p50", 50), ("p90", 90), ("max", 100))},
                "idle_frac": round(float((span - end).sum() / (len(end) * span)), 4),
                "tiles": [int(tiles.min()), int(tiles.max())], "per_xcc": per_xcc}

    if args.timed:
        for t, y, ns in geos:
            gx = max(1, t // y)
            nw = gx * y * 4
            st = torch.zeros(nw * 3, dtype=torch.int64, device="cuda")  # {t0, t1, xcc | tiles << 32}
            for it in range(args.timed if need == 8 else 0):  # the stamped static walk is built for k = 8
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                rc = lib.av_launch_timed(buf.data_ptr(), d_ptr, total * SS, SS, oo, SS, c_t.data_ptr(), ii.data_ptr(),
                                         oi.data_ptr(), L, nobj, r, gx, y, ctypes.c_void_p(s.cuda_stream), ns,
                                         st.data_ptr())
                assert rc == 0, rc
                b.record(s)
                torch.cuda.synchronize()
                if it == args.timed - 1:
                    tails.append(tail_report("pipe U3 (stamped)", (t, y, ns), a.elapsed_time(b),
                                             st.view(nw, 3).cpu().numpy()))
            for v in QUEUE:
                st = torch.zeros(t * 4 * 3, dtype=torch.int64, device="cuda")
                stamp_ptr[0] = st.data_ptr()
                for it in range(args.timed):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(s)
                    launch(v, gx, y, ns)
                    b.record(s)
                    torch.cuda.synchronize()
                    if it == args.timed - 1:
                        tails.append(tail_report(VARIANTS[v] + " (stamped)", (t, y, ns), a.elapsed_time(b),
                                                 st.view(t * 4, 3).cpu().numpy()))
                stamp_ptr[0] = None
            if need != 8:
                continue
            view().zero_()
            launch(15, 4, 8, ns)
            torch.cuda.synchronize()
            good = view().clone()
            view().zero_()
            rc = lib.av_launch_timed(buf.data_ptr(), d_ptr, total * SS, SS, oo, SS, c_t.data_ptr(), ii.data_ptr(),
                                     oi.data_ptr(), L, nobj, r, 1, 8, ctypes.c_void_p(s.cuda_stream), ns,
                                     torch.zeros(8 * 4 * 3, dtype=torch.int64, device="cuda").data_ptr())
            torch.cuda.synchronize()
            if not torch.equal(view(), good):
                bad.append(("timed", ns))
    rows = []
    for (v, (t, y, ns)), ts in times.items():
        med = statistics.median(ts)
        rows.append({"variant": VARIANTS[v], "blocks": t, "objects_in_flight": y, "nseg": ns, "ms": round(med, 3),
                     "GBps": round(alg / (med * 1e-3) / 1e9, 1)})
    rows.sort(key=lambda x: -x["GBps"])
    return {"separate": int(args.separate if args.separate >= 0 else separate), "bad_variants": bad,
            "top": rows[:12], "all": rows, "tails": tails}


if __name__ == "__main__":
    main()
