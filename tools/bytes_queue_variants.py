#!/usr/bin/env python3
"""A/B the unroll (U) and unit size (C) of the fused byte encode's first pass
(encode_bytes_queue_kernel, mapping 0, no switch record) at C3 (8/12, 128 x
256 MiB) and C5 (10/14, 16 x 1 GiB, 256 B chunk stride), in one process on one
allocation per shape; every variant's parity is compared with the product
variant's.  Median kernel ms and GB/s on the algorithmic bytes 4L(k+r).

    hipcc ... -shared -o tools/libbqvar.so tools/bytes_queue_variants.hip
    python tools/bytes_queue_variants.py [--rounds 5 --blocks 256,512]
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

NAMES = {0: "K8 U2 C3 (product)", 1: "K8 U3 C2", 2: "K8 U4 C2", 6: "K8 U1 C6",
         3: "K10 U1 C6 (product)", 4: "K10 U2 C3", 5: "K10 U3 C2", 7: "K4 U2 C3 (product)", 8: "K4 U4 C2",
         9: "K4 U3 C2"}
SHAPES = {"c3": (8, 12, 256, 128, 1, [0, 1, 2, 6]), "c5": (10, 14, 1024, 16, 256, [3, 4, 5]),
          "c2": (4, 6, 64, 32, 1, [7, 8, 9])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--blocks", type=str, default="256")
    ap.add_argument("--shapes", type=str, default="c5,c3")
    ap.add_argument("--switch", type=str, default="0,1", help="0: no switch record; 1: the product's switching pass")
    ap.add_argument("--variants-c5", type=str, default="", help="override the shape's variant list")
    ap.add_argument("--variants-c3", type=str, default="")
    ap.add_argument("--variants-c2", type=str, default="")
    ap.add_argument("--redo-blocks", type=str, default="",
                    help="instead: time the product's second pass (redo list + redo kernel) on these grids")
    args = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libbqvar.so"))
    lib.bqv_encode.restype = ctypes.c_int
    lib.bqv_encode.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                               ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32] + [ctypes.c_void_p] * 4 + \
        [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    lib.bqv_redo.restype = ctypes.c_int
    lib.bqv_redo.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                             ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32] + [ctypes.c_void_p] * 7 + \
        [ctypes.c_uint32, ctypes.c_void_p]
    s = torch.cuda.current_stream()
    ticket = torch.zeros(lib.bqv_ticket_words(), dtype=torch.int32, device="cuda")
    out = {}
    for shape in args.shapes.split(","):
        need, total, mib, nobj, align, variants = SHAPES[shape]
        over = getattr(args, f"variants_{shape}")
        if over:
            variants = [int(x) for x in over.split(",")]
        S = mib << 20
        L, cs, slot = D.slot_geometry(S, need, total, chunk_align=align)
        rows = total - need
        slots = D.device_empty(nobj * slot, torch.uint8)
        D.fill_symbols(slots.view(torch.int32), 11)
        coeff = np.zeros((rows, 16), dtype=np.uint32)
        coeff[:, :need] = D.Plan.encode(need, total).coefficients()
        c_t = torch.from_numpy(coeff.view(np.int32).reshape(-1)).cuda()
        oi = torch.arange(rows, dtype=torch.int32, device="cuda")
        flags = torch.zeros(nobj, dtype=torch.int32, device="cuda")
        par = slots.view(nobj, total, cs)[:, need:, : 4 * L]
        alg = nobj * 4 * L * total

        record = torch.zeros(nobj * (1 << 20), dtype=torch.uint8, device="cuda")

        def run(v, blocks, sw=0):
            flags.zero_()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            rc = lib.bqv_encode(v, slots.data_ptr(), slot, cs, L, S, nobj, rows, c_t.data_ptr(), oi.data_ptr(),
                                flags.data_ptr(), ticket.data_ptr(), blocks,
                                ctypes.c_void_p(record.data_ptr() if sw else 0), ctypes.c_void_p(s.cuda_stream))
            b.record(s)
            torch.cuda.synchronize()
            assert rc == 0, (v, rc)
            return a.elapsed_time(b)

        if args.redo_blocks:
            out[shape] = redo_ab(args, lib, s, ticket, shape, variants[0], slots, slot, cs, L, S, nobj, rows, c_t, oi,
                                 flags, record, par, alg)
            del slots, par
            torch.cuda.empty_cache()
            continue
        run(variants[0], 256)
        ref = par.clone()
        times = {}
        for r in range(args.rounds + 1):
            for v in variants:
                for blocks in (int(x) for x in args.blocks.split(",")):
                    for sw in (int(x) for x in args.switch.split(",")):
                        par.fill_(0)
                        ms = run(v, blocks, sw)
                        if not sw:  # the switching pass writes 1<<31 units of some objects
                            assert torch.equal(par, ref), (shape, v, blocks)
                        if r:
                            times.setdefault(f"{NAMES[v]} b{blocks}{' switch' if sw else ''}", []).append(ms)
        res = {}
        for k, ts in times.items():
            med = statistics.median(ts)
            res[k] = {"ms": round(med, 4), "gbs": round(alg / med / 1e6, 1), "min_ms": round(min(ts), 4)}
            print(f"{shape} {k}: {med:.4f} ms  {alg / med / 1e6:.1f} GB/s", flush=True)
        out[shape] = res
        del slots, par, ref
        torch.cuda.empty_cache()
    print(json.dumps(out))


def redo_ab(args, lib, s, ticket, shape, v, slots, slot, cs, L, S, nobj, rows, c_t, oi, flags, record, par, alg):
    """First pass with the switch record (not timed), mapping selection as
    select_mapping_kernel (rs_bytes.hip), then the second pass timed per grid;
    the final chunks must not depend on the grid."""
    status = torch.zeros(nobj, dtype=torch.int32, device="cuda")
    mapping = torch.zeros(nobj, dtype=torch.int32, device="cuda")
    lst = torch.zeros(nobj * (1 << 20) // 4, dtype=torch.int32, device="cuda")
    count = torch.zeros(1, dtype=torch.int32, device="cuda")
    ref, times = None, {}
    for r in range(args.rounds + 1):
        for blocks in (int(x) for x in args.redo_blocks.split(",")):
            flags.zero_()
            rc = lib.bqv_encode(v, slots.data_ptr(), slot, cs, L, S, nobj, rows, c_t.data_ptr(), oi.data_ptr(),
                                flags.data_ptr(), ticket.data_ptr(), 512, ctypes.c_void_p(record.data_ptr()),
                                ctypes.c_void_p(s.cuda_stream))
            assert rc == 0
            f = flags
            zero_ok, high_ok = (f & 1) == 0, (f & 2) == 0
            mapping.copy_(torch.where(zero_ok, 0, torch.where(high_ok, -2**31, 0)).to(torch.int32))
            status.copy_((~zero_ok & ~high_ok).to(torch.int32))
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            rc = lib.bqv_redo(v, slots.data_ptr(), slot, cs, L, S, nobj, rows, c_t.data_ptr(), oi.data_ptr(),
                              mapping.data_ptr(), status.data_ptr(), record.data_ptr(), lst.data_ptr(), count.data_ptr(),
                              blocks, ctypes.c_void_p(s.cuda_stream))
            b.record(s)
            torch.cuda.synchronize()
            assert rc == 0
            ok = (status == 0).nonzero().flatten()  # objects needing the random fallback are not final
            if ref is None:
                ref = par[ok].clone()
            else:
                assert torch.equal(par[ok], ref), (shape, blocks)
            if r:
                times.setdefault(f"redo b{blocks}", []).append(a.elapsed_time(b))
    res = {"switched": int((mapping != 0).sum().item()), "listed_units": int(count.item())}
    for k, ts in times.items():
        res[k] = {"ms": round(statistics.median(ts), 4), "min_ms": round(min(ts), 4)}
        print(f"{shape} {k}: {res[k]['ms']:.4f} ms", flush=True)
    return res


if __name__ == "__main__":
    main()
