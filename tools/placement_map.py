#!/usr/bin/env python3
"""Is the slow placement mode spread over a whole buffer or a property of
some of its objects?  Same allocation sequence as tools/placement_probe.py
(C3 buffers of 128 objects x 12 shards x 8 Mi symbols), then, per buffer:
the product encode over the whole batch, and per object the encode's
traffic mix (read 8 + write 4 stripes, XOR math) and a write-only 4-stripe
mix with the whole grid on that one object; then the product kernel
(tools/apply_variants.hip variant 8) over the whole batch with 1..128 objects
in flight (grid 512/y x y).

    make placeprobe && python tools/placement_map.py [--buffers 5]
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

import torch  # noqa: E402  (owns the HIP runtime; load before our .so)

from slime_amd import device as D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--buffers", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libplaceprobe.so"))
    lib.pp_launch.restype = ctypes.c_int
    lib.pp_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                              ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    need, total, L, nobj = 8, 12, 8 << 20, 128
    lay = D.layout_of(total, L)
    enc = D.Plan.encode(need, total)
    sink = torch.empty(512 * 256, dtype=torch.int32, device="cuda")
    av = ctypes.CDLL(os.path.join(ROOT, "tools", "libapplyvar.so"))
    av.av_launch.restype = ctypes.c_int
    av.av_launch.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_uint64] * 4 + \
        [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
    import numpy as np
    coeff = np.zeros((total - need, 16), dtype=np.uint32)
    coeff[:, :need] = enc.coefficients()
    c_t = torch.from_numpy(coeff.view(np.int32).reshape(-1)).cuda()
    ii = torch.arange(need, dtype=torch.int32, device="cuda")
    oi = torch.arange(need, total, dtype=torch.int32, device="cuda")
    bufs = []
    for b in range(args.buffers):
        free, _ = torch.cuda.mem_get_info()
        if free < nobj * total * L * 4 + (8 << 30):
            break
        t = torch.empty(nobj * total * L, dtype=torch.int32, device="cuda")
        D.fill_symbols(t, b + 1)
        bufs.append(t)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()

    def timed(fn):
        fn()
        ts = []
        for _ in range(args.reps):
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            fn()
            e.record(s)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(e))
        return statistics.median(ts)

    out = []
    for b, t in enumerate(bufs):
        ms = timed(lambda: enc(t, lay, t, lay, L, nobj, dst_offset=need * L))
        row = {"buffer": b, "va": hex(t.data_ptr()), "encode_GBps": round(nobj * L * 4 * total / (ms * 1e-3) / 1e9, 1)}
        for mix, name, nstripes in ((3, "r8w4", 12), (2, "w4", 4)):
            per = []
            for o in range(nobj):
                ptr = t.data_ptr() + o * total * L * 4

                def go(mix=mix, ptr=ptr):
                    assert lib.pp_launch(mix, ptr, total * L, L, L, 1, 512, 1, sink.data_ptr(),
                                         ctypes.c_void_p(s.cuda_stream), 1) == 0
                per.append(round(L * 4 * nstripes / (timed(go) * 1e-3) / 1e9))
            row[name] = {"median": statistics.median(per), "min": min(per), "max": max(per), "per_object": per}
        for gy in (1, 2, 8, 32, 128):
            def prod(gy=gy):
                assert av.av_launch(8, need, t.data_ptr(), t.data_ptr(), total * L, L, total * L, L, c_t.data_ptr(),
                                    ii.data_ptr(), oi.data_ptr(), L, nobj, total - need, max(1, 512 // gy), gy,
                                    ctypes.c_void_p(s.cuda_stream), 1) == 0
            row[f"product_inflight{gy}_GBps"] = round(nobj * L * 4 * total / (timed(prod) * 1e-3) / 1e9, 1)
        out.append(row)
        print(json.dumps({k: (v if not isinstance(v, dict) else {kk: vv for kk, vv in v.items() if kk != "per_object"})
                          for k, v in row.items()}), flush=True)
    print(json.dumps({"per_buffer": out}))


if __name__ == "__main__":
    main()
