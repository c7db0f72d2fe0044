#!/usr/bin/env python3
"""Time the five-K-step matrix-core apply variants (tools/wide_variants.hip)
on one encode shape in interleaved rounds in one process; every variant's
parity is compared bit-exact with variant 0.

    make widevar && python tools/wide_variants.py --need 80 --total 100 --mib 256 --nobj 32
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--need", type=int, default=80)
    ap.add_argument("--total", type=int, default=100)
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--nobj", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--variants", default="0,2,5,6,7")
    a = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libwidevar.so"))
    lib.wv_name.restype = ctypes.c_char_p
    lib.wv_table.restype = ctypes.c_uint64
    lib.wv_table.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                             ctypes.c_uint64]
    lib.wv_launch.restype = ctypes.c_int
    lib.wv_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_uint64] * 4 + \
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
         ctypes.c_void_p]
    k, rows = a.need, a.total - a.need
    L = ((a.mib << 20) // 4 + k - 1) // k
    L -= L % 128  # whole tiles (the harness has no column tail)
    stride = L  # a multiple of 64 symbols
    obj = stride * a.total
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    buf = torch.randint(-2**31, 2**31 - 5, (a.nobj * obj,), dtype=torch.int32, device=dev, generator=g)
    c = np.ascontiguousarray((np.random.default_rng(7).integers(0, 0xFFFFFFFB, rows * k, dtype=np.uint64))
                             .astype(np.uint32))
    tables = {}
    for form in (0, 4):  # the 16x16 table, the 32x32 table
        n = lib.wv_table(form, c.ctypes.data, rows, k, None, 0)
        host = np.zeros(n, dtype=np.uint8)
        lib.wv_table(form, c.ctypes.data, rows, k, host.ctypes.data, n)
        tables[form] = torch.from_numpy(host).to(dev)
    out_idx = torch.arange(k, a.total, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    variants = [int(v) for v in a.variants.split(",")]

    def launch(v):
        table = tables[4 if 4 <= v <= 7 else 0]
        rc = lib.wv_launch(v, buf.data_ptr(), buf.data_ptr(), obj, stride, obj, stride, table.data_ptr(),
                           out_idx.data_ptr(), L, a.nobj, rows, k, sp)
        if rc:
            raise SystemExit(f"variant {v}: hip error {rc}")

    parity = buf.view(a.nobj, a.total, stride)[:, k:, :]
    launch(0)
    ref = parity.clone()
    ok = {}
    for v in variants:
        parity.zero_()
        launch(v)
        torch.cuda.synchronize()
        ok[v] = bool(torch.equal(parity, ref)) if v != 8 else None  # 8: another layout, timing only
    times = {v: [] for v in variants}
    for r in range(a.rounds):
        for v in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            launch(v)
            e1.record(stream)
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1))
    alg = a.nobj * 4 * L * a.total
    for v in variants:
        med = statistics.median(times[v][1:] if len(times[v]) > 2 else times[v])
        print(json.dumps({"variant": v, "name": lib.wv_name(v).decode(), "need": k, "total": a.total,
                          "ms": round(med, 4), "min": round(min(times[v]), 4), "frac": round(alg / med / 1e-3 / 8e12, 4),
                          "exact_vs_v0": ok[v]}), flush=True)


if __name__ == "__main__":
    main()
