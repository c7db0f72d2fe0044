#!/usr/bin/env python3
"""Read bandwidth by working-set size (tools/ubench.hip read kernels): sizes that
fit the 256 MB Infinity Cache (MALL) against ones that stream from HBM, plus
write and copy at HBM scale.  Run beside the placement probe to see whether a
slow-placement box differs in its cache or only in its DRAM.

    make ubench && python tools/mall_probe.py
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (owns the HIP runtime; load before our .so)

lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libubench.so"))
V, U64, U32, I = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
for name, args in {"ub_read": [V, V, U64, U32, I], "ub_read_nt": [V, V, U64, U32, I],
                   "ub_write": [V, U64, U32, I], "ub_copy": [V, V, U64, U32, I]}.items():
    getattr(lib, name).argtypes = args
    getattr(lib, name).restype = ctypes.c_float
assert lib.ub_init() == 0


def main():
    mib = 1 << 20
    big = torch.empty((16 << 30) // 4, dtype=torch.int32, device="cuda")
    big.fill_(1)
    sink = torch.empty(1 << 24, dtype=torch.int32, device="cuda")
    out = {}
    for size_mib in (32, 64, 128, 192, 512, 2048, 8192):
        n16 = size_mib * mib // 16
        ms = lib.ub_read(big.data_ptr(), sink.data_ptr(), n16, 2048, 20)
        out[f"read_{size_mib}MiB_GBps"] = round(size_mib * mib / (ms * 1e-3) / 1e9, 1)
    n16 = 8192 * mib // 16
    out["read_nt_8GiB_GBps"] = round(8192 * mib / (lib.ub_read_nt(big.data_ptr(), sink.data_ptr(), n16, 8192, 5)
                                                  * 1e-3) / 1e9, 1)
    out["write_8GiB_GBps"] = round(8192 * mib / (lib.ub_write(big.data_ptr(), n16, 2048, 5) * 1e-3) / 1e9, 1)
    half = n16 // 2
    out["copy_8GiB_GBps"] = round(2 * half * 16 / (lib.ub_copy(big.data_ptr(), big.data_ptr() + half * 16, half,
                                                               2048, 5) * 1e-3) / 1e9, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
