#!/usr/bin/env python3
"""Measurement helpers for DESIGN.md (not the benchmark of record; see bench.py).

  copy      practical HBM peak: device-to-device copy of a buffer >> 256 MiB MALL
  compute   VALU ceiling of the apply kernel: small, cache-resident batches
            re-run back to back (no HBM traffic after the first pass)
  shapes    device-resident encode/decode GiB/s for BASELINE configs C2..C5
  e2e       host memory -> device -> host rate of the Go-API entry point
            (CreateParities on pageable numpy buffers, PCIe-inclusive)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from slime_amd import device as D  # noqa: E402

GIB = 1 << 30


def timed(fn, iters, stream):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    a.record(stream)
    for _ in range(iters):
        fn()
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def copy_peak():
    n = 4 * GIB // 4
    src = torch.empty(n, dtype=torch.int32, device="cuda")
    dst = torch.empty_like(src)
    ms = timed(lambda: dst.copy_(src), 10, torch.cuda.current_stream())
    return {"copy_GBps": round(2 * n * 4 / (ms * 1e-3) / 1e9, 1), "bytes_moved": 2 * n * 4}


def run_shape(need, total, obj_mib, nobj, erase, iters=5):
    S = obj_mib << 20
    L = -(-(-(-S // 4)) // need)
    lay = D.layout_of(total, L)
    buf = torch.empty(nobj * total * L, dtype=torch.int32, device="cuda")
    D.fill_symbols(buf, 99)
    enc = D.Plan.encode(need, total)
    have = [i for i in range(total) if i not in erase][:need]
    dec = D.Plan.reconstruct(need, total, have, erase)
    rec = torch.empty(nobj * len(erase) * L, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    e_ms = timed(lambda: enc(buf, lay, buf, lay, L, nobj, dst_offset=need * L), iters, s)
    d_ms = timed(lambda: dec(buf, lay, rec, D.layout_of(len(erase), L), L, nobj), iters, s)
    enc_b = nobj * 4 * L * total
    dec_b = nobj * 4 * L * (need + len(erase))
    out = {"need": need, "total": total, "object_mib": obj_mib, "nobj": nobj, "erase": erase,
           "encode_ms": round(e_ms, 4), "decode_ms": round(d_ms, 4),
           "encode_obj_GiBps": round(nobj * S / GIB / (e_ms * 1e-3), 1),
           "decode_obj_GiBps": round(nobj * S / GIB / (d_ms * 1e-3), 1),
           "encode_hbm_GBps": round(enc_b / (e_ms * 1e-3) / 1e9, 1),
           "decode_hbm_GBps": round(dec_b / (d_ms * 1e-3) / 1e9, 1)}
    del buf, rec
    torch.cuda.empty_cache()
    return out


def compute_ceiling():
    # 8/12 on 64 objects x 256 KiB: 24 MiB working set, L2/MALL resident.
    res = run_shape(8, 12, 1, 16, [0, 1, 2, 3], iters=200)
    res["note"] = "cache-resident (16 x 1 MiB objects): VALU/issue ceiling, not HBM"
    return res


def e2e(need=8, total=12, obj_mib=64):
    import numpy as np

    from slime_amd import rs
    L = (obj_mib << 20) // 4 // need
    rng = np.random.default_rng(1)
    data = [rng.integers(0, 4294967291, size=L, dtype=np.uint64).astype(np.uint32) for _ in range(need)]
    rs.CreateParities(data, total)
    t0 = time.perf_counter()
    it = 3
    for _ in range(it):
        rs.CreateParities(data, total)
    dt = (time.perf_counter() - t0) / it
    return {"e2e_encode_obj_GiBps": round(need * L * 4 / GIB / dt, 3), "object_mib": obj_mib,
            "path": "pageable numpy -> hipMemcpyAsync H2D -> kernel -> D2H, one object per call"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="*", default=["copy", "compute", "shapes", "e2e"])
    args = ap.parse_args()
    out = {}
    if "copy" in args.what:
        out["copy"] = copy_peak()
    if "compute" in args.what:
        out["compute"] = compute_ceiling()
    if "shapes" in args.what:
        out["shapes"] = [
            run_shape(4, 6, 64, 32, [0, 1]),              # C2
            run_shape(8, 12, 256, 128, [0, 1, 2, 3]),    # C3 / C4
            run_shape(8, 12, 256, 128, [0, 3, 8, 11]),   # C4 mixed
            run_shape(8, 12, 512, 32, [0, 1, 2, 3]),     # 64 MiB shards (target text)
            run_shape(10, 14, 1024, 16, [0, 1, 2, 3]),   # C5 per-GPU slice (8 of 64 at G=8 -> 16 here)
            run_shape(2, 3, 64, 64, [0]),
        ]
    if "e2e" in args.what:
        out["e2e"] = e2e()
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
