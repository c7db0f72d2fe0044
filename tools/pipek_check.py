#!/usr/bin/env python3
"""Bit-exactness of the k-template pipelined kernel at k > 16 (harness
av_launch_pipek) against the C oracle, on small shapes, with mismatch
locations: which output rows, which columns.

    make applyvar && python tools/pipek_check.py
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle_c as OC  # noqa: E402
from slime_amd import device as D  # noqa: E402


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libapplyvar.so"))
    lib.av_launch_pipek.restype = ctypes.c_int
    lib.av_launch_pipek.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_uint64] * 4 + \
        [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
    out = []
    for K, U in ((20, 1), (20, 2), (24, 1), (24, 2), (28, 1), (32, 1)):
        for rows in (1, 4, 8):
            for L in (64 * 4, 4099, 65536):
                total = K + rows
                nobj = 2
                buf = torch.empty(nobj * total * L, dtype=torch.int32, device="cuda")
                D.fill_symbols(buf, K * 100 + rows)
                torch.cuda.synchronize()
                h = buf.cpu().numpy().view(np.uint32).reshape(nobj, total, L).copy()
                pm = OC.parity_matrix(K, rows)[K:]
                cs = -(-K // 16) * 16
                coeff = np.zeros((rows, cs), dtype=np.uint32)
                coeff[:, :K] = pm
                c_t = torch.from_numpy(coeff.view(np.int32).reshape(-1)).cuda()
                ii = torch.arange(K, dtype=torch.int32, device="cuda")
                oi = torch.arange(K, K + rows, dtype=torch.int32, device="cuda")
                s = torch.cuda.current_stream()
                rc = lib.av_launch_pipek(K, U, buf.data_ptr(), buf.data_ptr(), total * L, L, total * L, L,
                                         c_t.data_ptr(), ii.data_ptr(), oi.data_ptr(), L, nobj, rows, 4, 2,
                                         ctypes.c_void_p(s.cuda_stream), 1)
                assert rc == 0, rc
                torch.cuda.synchronize()
                got = buf.cpu().numpy().view(np.uint32).reshape(nobj, total, L)
                bad_rows, bad_cols = set(), []
                for o in range(nobj):
                    ref = OC.apply_matrix(pm, [h[o, j] for j in range(K)])
                    for i in range(rows):
                        d = np.nonzero(got[o, K + i] != ref[i])[0]
                        if d.size:
                            bad_rows.add(i)
                            bad_cols.extend(d[:4].tolist())
                out.append({"K": K, "U": U, "rows": rows, "L": L, "ok": not bad_rows, "bad_rows": sorted(bad_rows),
                            "first_bad_cols": bad_cols[:8]})
                print(json.dumps(out[-1]), flush=True)
                del buf


if __name__ == "__main__":
    main()
