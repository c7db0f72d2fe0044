#!/usr/bin/env python3
"""A/B of the byte encode's second pass: the product's re-encode of the units
a switched object encoded with mapping 0, against a parity correction from
top bits the first pass stored (tools/topbits_fix.hip, the product
kernels).  In one process on one
allocation per shape, alternating: the first pass without / with the bit
store, then the redo list and the re-encode / the correction (plus the
edge-only redo).  The corrected chunks must equal the re-encoded ones on every
object MapToGF maps to 0 or 1<<31.  Prints per-variant median ms.

    make tools/libtopbits.so && python tools/topbits_fix.py [--shapes c5,c3 --rounds 6]
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

# shape: (tbf shape id, need, total, object MiB, objects, chunk alignment, blocks)
SHAPES = {"c5": (1, 10, 14, 1024, 16, 256, 512), "c3": (0, 8, 12, 256, 128, 256, 512)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="c5,c3")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--fix-blocks", default="512", help="grids of the correction kernel")
    args = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libtopbits.so"))
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    lib.tbf_pass0.argtypes = [i32, i32, vp, u64, u64, u64, u64, u32, u32, vp, vp, vp, vp, u32, vp, vp, vp]
    lib.tbf_second.argtypes = [i32, i32, vp, u64, u64, u64, u64, u32, u32, vp, vp, vp, vp, vp, vp, vp, vp, u32, vp]
    lib.tbf_bits_bytes.restype = u64
    lib.tbf_bits_bytes.argtypes = [i32, u64, u64, u32]
    lib.tbf_units.restype = u32
    lib.tbf_units.argtypes = [i32, u64, u64, u32]
    s = torch.cuda.current_stream()
    ticket = torch.zeros(lib.tbf_ticket_words(), dtype=torch.int32, device="cuda")
    out = {}
    for shape in args.shapes.split(","):
        sid, need, total, mib, nobj, align, blocks = SHAPES[shape]
        S = mib << 20
        L, cs, slot = D.slot_geometry(S, need, total, chunk_align=align)
        rows = total - need
        slots = D.device_empty(nobj * slot, torch.uint8)
        D.fill_symbols(slots.view(torch.int32), args.seed)
        coeff = np.zeros((rows, 16), dtype=np.uint32)
        coeff[:, :need] = D.Plan.encode(need, total).coefficients()
        c_t = torch.from_numpy(coeff.view(np.int32).reshape(-1)).cuda()
        oi = torch.arange(rows, dtype=torch.int32, device="cuda")
        flags = torch.zeros(nobj, dtype=torch.int32, device="cuda")
        mapping = torch.zeros(nobj, dtype=torch.int32, device="cuda")
        status = torch.zeros(nobj, dtype=torch.int32, device="cuda")
        units = lib.tbf_units(sid, S, L, nobj)
        record = torch.zeros(nobj * units, dtype=torch.uint8, device="cuda")
        lst = torch.zeros(nobj * units, dtype=torch.int32, device="cuda")
        count = torch.zeros(2, dtype=torch.int32, device="cuda")
        bits = torch.zeros(lib.tbf_bits_bytes(sid, S, L, nobj), dtype=torch.uint8, device="cuda")
        par = slots.view(nobj, slot)[:, need * cs: total * cs]
        alg0 = nobj * 4 * L * total  # the first pass's algorithmic bytes (interior ~ all)

        def run(fix: int, fblocks: int):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            flags.zero_()
            ev[0].record(s)
            assert lib.tbf_pass0(sid, fix, slots.data_ptr(), slot, cs, L, S, nobj, rows, c_t.data_ptr(),
                                 oi.data_ptr(), flags.data_ptr(), ticket.data_ptr(), blocks, record.data_ptr(),
                                 bits.data_ptr(), s.cuda_stream) == 0
            ev[1].record(s)
            zero_ok, high_ok = (flags & 1) == 0, (flags & 2) == 0
            mapping.copy_(torch.where(zero_ok, 0, torch.where(high_ok, -2**31, 0)).to(torch.int32))
            status.copy_((~zero_ok & ~high_ok).to(torch.int32))
            ev2 = torch.cuda.Event(enable_timing=True)
            ev2.record(s)
            assert lib.tbf_second(sid, fix, slots.data_ptr(), slot, cs, L, S, nobj, rows, c_t.data_ptr(),
                                  oi.data_ptr(), mapping.data_ptr(), status.data_ptr(), record.data_ptr(),
                                  bits.data_ptr(), lst.data_ptr(), count.data_ptr(), fblocks, s.cuda_stream) == 0
            ev[2].record(s)
            torch.cuda.synchronize()
            assert int(ticket.abs().sum().item()) == 0
            return ev[0].elapsed_time(ev[1]), ev2.elapsed_time(ev[2]), int(count[0].item())

        ok = None
        ref = None
        times = {}
        variants = [(0, blocks)] + [(1, int(b)) for b in args.fix_blocks.split(",")]
        for r in range(args.rounds + 1):
            for fix, fb in variants:
                t0, t1, listed = run(fix, fb)
                if ok is None:
                    ok = (status == 0).nonzero().flatten()
                    switched = int(((mapping != 0) & (status == 0)).sum().item())
                got = par[ok].clone()
                if ref is None:
                    ref = got
                else:
                    assert torch.equal(got, ref), (shape, fix, fb, "parity differs")
                del got
                if r:
                    key = "re-encode" if not fix else f"correction b{fb}"
                    times.setdefault(key, {"pass0": [], "second": [], "listed": []})
                    times[key]["pass0"].append(t0)
                    times[key]["second"].append(t1)
                    times[key]["listed"].append(listed)
        res = {"switched": switched, "nobj": nobj, "bits_bytes": bits.numel()}
        for k, v in times.items():
            p0, p1 = statistics.median(v["pass0"]), statistics.median(v["second"])
            res[k] = {"pass0_ms": round(p0, 4), "second_ms": round(p1, 4), "sum_ms": round(p0 + p1, 4),
                      "pass0_frac": round(alg0 / (p0 * 1e-3) / 8e12, 4),
                      "listed_median": int(statistics.median(v["listed"]))}
            print(shape, k, res[k], flush=True)
        out[shape] = res
        del slots, par, ref, bits
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
