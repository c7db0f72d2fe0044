#!/usr/bin/env python3
"""Run-to-run variance of the C3 encode/decode kernels across fresh device
allocations in one process (is the spread the allocation's physical layout,
or the kernel?).  Each round: allocate the 48 GiB object buffer, fill, time
encode + in-place repair (median of 5 each), free it back to the driver.

    python tools/alloc_variance.py [--rounds 6] [--inflight 0,16]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from slime_amd import device as D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--nobj", type=int, default=128)
    args = ap.parse_args()
    need, total, L, nobj = 8, 12, 8 << 20, args.nobj
    lay = D.layout_of(total, L)
    enc = D.Plan.encode(need, total)
    dec = D.Plan.reconstruct(need, total, list(range(4, 12)), [0, 1, 2, 3]).set_outputs([0, 1, 2, 3])
    s = torch.cuda.current_stream()
    out = []
    for r in range(args.rounds):
        pad = torch.empty((r % 3) * (1 << 28), dtype=torch.int32, device="cuda")  # shift the placement
        buf = torch.empty(nobj * total * L, dtype=torch.int32, device="cuda")
        D.fill_symbols(buf, r)
        times = {"enc": [], "dec": []}
        for _ in range(6):
            for name, fn in (("enc", lambda: enc(buf, lay, buf, lay, L, nobj, dst_offset=need * L)),
                             ("dec", lambda: dec(buf, lay, buf, lay, L, nobj))):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                fn()
                b.record(s)
                torch.cuda.synchronize()
                times[name].append(a.elapsed_time(b))
        out.append({"round": r, "pad_gib": (r % 3), "enc_ms": round(statistics.median(times["enc"][1:]), 3),
                    "dec_ms": round(statistics.median(times["dec"][1:]), 3),
                    "enc_all": [round(t, 2) for t in times["enc"]], "buf": hex(buf.data_ptr())})
        del buf, pad
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
