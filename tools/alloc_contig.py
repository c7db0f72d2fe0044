#!/usr/bin/env python3
"""Does physically contiguous device memory remove the slow-allocation mode of
the C3 encode?  Interleaved rounds of hipMalloc vs hipExtMallocWithFlags(
hipDeviceMallocContiguous), 48 GiB each, encode + in-place repair timed on the
raw C-ABI.

    python tools/alloc_contig.py [--rounds 6]
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

import torch  # noqa: E402

from slime_amd import _native as N  # noqa: E402
from slime_amd import device as D  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so.7")  # torch's runtime (already loaded: same soname)
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipFree.argtypes = [ctypes.c_void_p]
hip.hipDeviceSynchronize.argtypes = []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    args = ap.parse_args()
    need, total, L, nobj = 8, 12, 8 << 20, 128
    nbytes = nobj * total * L * 4
    lay = D.layout_of(total, L)
    enc = D.Plan.encode(need, total)
    dec = D.Plan.reconstruct(need, total, list(range(4, 12)), [0, 1, 2, 3]).set_outputs([0, 1, 2, 3])
    torch.cuda.init()
    s = torch.cuda.current_stream()
    res = []
    for r in range(args.rounds):
        for flag in (0, 4):
            p = ctypes.c_void_p()
            rc = hip.hipMalloc(ctypes.byref(p), nbytes) if flag == 0 else \
                hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, flag)
            if rc != 0:
                res.append({"round": r, "flag": flag, "error": rc})
                continue
            N.check(N.lib.slime_rs_fill_symbols(0, p, nbytes // 4, r, ctypes.c_void_p(s.cuda_stream)))
            times = {"enc": [], "dec": []}
            for _ in range(5):
                for name, plan, dst in (("enc", enc, p.value + need * L * 4), ("dec", dec, p.value)):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(s)
                    N.check(N.lib.slime_rs_plan_execute(plan._h, p, lay, ctypes.c_void_p(dst), lay, L, nobj,
                                                        ctypes.c_void_p(s.cuda_stream)))
                    b.record(s)
                    torch.cuda.synchronize()
                    times[name].append(a.elapsed_time(b))
            res.append({"round": r, "flag": flag, "enc_ms": round(statistics.median(times["enc"]), 3),
                        "dec_ms": round(statistics.median(times["dec"]), 3), "ptr": hex(p.value)})
            hip.hipFree(p)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
