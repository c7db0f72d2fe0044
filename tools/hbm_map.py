#!/usr/bin/env python3
"""Map streaming bandwidth across device memory: allocate consecutive 8 GiB
buffers until ~90% of HBM is taken and time a 16 B/lane read and copy kernel
(tools/ubench.hip) on each.  Shows whether some placements are slower.

    make ubench && python tools/hbm_map.py
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libubench.so"))
V, U64, U32, I = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
lib.ub_read.argtypes = [V, V, U64, U32, I]
lib.ub_read.restype = ctypes.c_float
lib.ub_copy.argtypes = [V, V, U64, U32, I]
lib.ub_copy.restype = ctypes.c_float
assert lib.ub_init() == 0

GIB = 1 << 30


def main():
    free, total = torch.cuda.mem_get_info()
    piece = 8 * GIB
    n16 = piece // 16
    sink = torch.empty(1 << 24, dtype=torch.int32, device="cuda")
    bufs, rows = [], []
    while free - piece > total // 10:
        b = torch.empty(piece // 4, dtype=torch.int32, device="cuda")
        b.fill_(1)
        ms_r = lib.ub_read(b.data_ptr(), sink.data_ptr(), n16, 2048, 3)
        half = n16 // 2
        ms_c = lib.ub_copy(b.data_ptr(), b.data_ptr() + half * 16, half, 2048, 3)
        rows.append({"i": len(bufs), "va": hex(b.data_ptr()), "read_GBps": round(piece / (ms_r * 1e-3) / 1e9, 1),
                     "copy_GBps": round(2 * half * 16 / (ms_c * 1e-3) / 1e9, 1)})
        bufs.append(b)
        free, _ = torch.cuda.mem_get_info()
    print(json.dumps({"total_GiB": round(total / GIB, 1), "pieces": rows}, indent=1))


if __name__ == "__main__":
    main()
