#!/usr/bin/env python3
"""Driver for tools/ubench.hip: HBM ceilings for the apply kernel's access
pattern and its VALU ceiling ("What bounds the kernel").

    make ubench && python tools/ubench.py
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (owns the HIP runtime; load before our .so)

lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libubench.so"))
V, U64, U32, I = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
for name, args in {
    "ub_copy": [V, V, U64, U32, I], "ub_read": [V, V, U64, U32, I], "ub_read_nt": [V, V, U64, U32, I],
    "ub_read_glds": [V, V, U64, U32, I, I], "ub_write": [V, U64, U32, I],
    "ub_pattern8": [V, V, U64, U64, U64, U64, U64, U32, U32, U32, I],
    "ub_compute8": [V, V, U64, U32, U32, I], "ub_mad": [V, U64, U32, I],
}.items():
    getattr(lib, name).argtypes = args
    getattr(lib, name).restype = ctypes.c_float
assert lib.ub_init() == 0

GIB = 1 << 30
CUS, CLK = 256, 2.4e9


def gbps(nbytes, ms):
    return round(nbytes / (ms * 1e-3) / 1e9, 1)


def main():
    out = {}
    torch.cuda.init()
    n = 8 * GIB // 16
    a = torch.empty(n * 4, dtype=torch.int32, device="cuda")
    b = torch.empty(n * 4, dtype=torch.int32, device="cuda")
    a.fill_(1)
    for grid in (2048, 8192, 32768):
        out[f"copy_grid{grid}"] = gbps(2 * n * 16, lib.ub_copy(a.data_ptr(), b.data_ptr(), n, grid, 5))
        out[f"read_grid{grid}"] = gbps(n * 16, lib.ub_read(a.data_ptr(), b.data_ptr(), n, grid, 5))
        out[f"read_nt_grid{grid}"] = gbps(n * 16, lib.ub_read_nt(a.data_ptr(), b.data_ptr(), n, grid, 5))
        out[f"read_glds_grid{grid}"] = gbps(n * 16, lib.ub_read_glds(a.data_ptr(), b.data_ptr(), n, grid, 0, 5))
        out[f"read_glds_nt_grid{grid}"] = gbps(n * 16, lib.ub_read_glds(a.data_ptr(), b.data_ptr(), n, grid, 1, 5))
        out[f"write_grid{grid}"] = gbps(n * 16, lib.ub_write(b.data_ptr(), n, grid, 5))
    del a, b
    torch.cuda.empty_cache()
    # Apply-kernel pattern: 128 objects x 12 shards x 8Mi symbols (C3 layout),
    # in place (reads shards 0..7, writes 8..11), optionally padded shards.
    L, nobj, total, maxpad = 8 << 20, 128, 12, 4096 + 64
    big = torch.empty(nobj * total * (L + maxpad), dtype=torch.int32, device="cuda")
    for pad in (0, 64, maxpad):
        ss = L + pad
        assert nobj * total * ss <= big.numel()  # host-side bound before a raw launch
        for gx in (8, 16, 32, 64):
            ms = lib.ub_pattern8(big.data_ptr(), big.data_ptr() + 8 * ss * 4, total * ss, ss, total * ss, ss, L,
                                 nobj, 4, gx, 3)
            out[f"pattern8r4_pad{pad}_gx{gx}"] = gbps(nobj * L * 4 * 12, ms)
    del big
    torch.cuda.empty_cache()
    # VALU ceiling of the 8-input, 4-row math (no memory traffic).
    coeff = torch.randint(0, 2**31 - 1, (64,), dtype=torch.int32, device="cuda")
    sink = torch.empty(1 << 22, dtype=torch.int32, device="cuda")
    for grid in (2048, 4096):
        iters = 256
        ms = lib.ub_compute8(coeff.data_ptr(), sink.data_ptr(), iters, 4, grid, 3)
        cols = grid * 256 * iters * 4
        out[f"compute8r4_grid{grid}_Gcols_per_s"] = round(cols / (ms * 1e-3) / 1e9, 1)
        # HBM-equivalent: each column moves 48 B at 8/12 encode.
        out[f"compute8r4_grid{grid}_equiv_GBps"] = gbps(cols * 48, ms)
    ms = lib.ub_mad(sink.data_ptr(), 1024, 4096, 3)
    mads = 4096 * 256 * 1024 * 8
    out["mac_per_s_T"] = round(mads / (ms * 1e-3) / 1e12, 3)
    out["mac_lane_ops_per_clk_per_CU"] = round(mads / (ms * 1e-3) / CLK / CUS, 2)
    out["note_mac"] = "one MAC = v_mad_u64_u32 + v_addc_co_u32 (mac4); full-rate VALU = 128 lane-ops/clk/CU"
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    np.random.seed(0)
    main()
